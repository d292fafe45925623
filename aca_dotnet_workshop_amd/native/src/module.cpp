// Python bindings for the native state-store and broker engines (`_ttnative`).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include "apphost.hpp"
#include "backingfront.hpp"
#include "broker.hpp"
#include "docstore.hpp"
#include "httpparse.hpp"

namespace py = pybind11;
using namespace tt;

// Lower-cased header list -> dict; repeated headers joined by ", " except set-cookie (a list).
template <class List>
static py::dict headers_dict(const List& headers) {
  py::dict hd;
  for (auto& [k, v] : headers) {
    py::str key(k);
    if (hd.contains(key)) {
      if (k == "set-cookie") {
        py::object prev = hd[key];
        py::list l;
        if (py::isinstance<py::list>(prev)) l = prev.cast<py::list>();
        else l.append(prev);
        l.append(py::str(v));
        hd[key] = l;
      } else {
        hd[key] = py::str(hd[key].cast<std::string>() + ", " + v);
      }
    } else {
      hd[key] = py::str(v);
    }
  }
  return hd;
}

// [(name, value), ...] from Python -> header list with lower-cased names (framing headers are
// filtered by the writer, which compares lower-case names).
static ev::HeaderList header_list(const py::handle& seq) {
  ev::HeaderList out;
  for (auto item : seq) {
    auto t = item.cast<py::tuple>();
    std::string k = t[0].cast<std::string>();
    for (auto& ch : k) ch = (char)std::tolower((unsigned char)ch);
    out.emplace_back(std::move(k), py::str(t[1]).cast<std::string>());  // any value, like f"{v}"
  }
  return out;
}

static std::string bytes_of(const py::handle& b) {
  char* p;
  Py_ssize_t n;
  if (PyBytes_AsStringAndSize(b.ptr(), &p, &n) != 0) throw py::error_already_set();
  return std::string(p, (size_t)n);
}

PYBIND11_MODULE(_ttnative, m) {
  m.doc() = "Native document store + message broker engines (C++17)";

  static py::exception<EtagMismatch> etag_exc(m, "EtagMismatch");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const EtagMismatch& e) {
      PyErr_SetString(etag_exc.ptr(), e.what());
    } catch (const QueryError& e) {
      PyErr_SetString(PyExc_ValueError, e.what());
    } catch (const ParseError& e) {
      PyErr_SetString(PyExc_ValueError, (std::string("invalid JSON: ") + e.what()).c_str());
    }
  });

  // (start-line a, b, c, headers dict) with lower-cased names; repeated headers joined by
  // ", " except set-cookie, which becomes a list.  Raises ValueError on malformed input.
  m.def("parse_http_head", [](py::bytes raw) {
    std::string_view sv = raw;
    HttpHead h;
    try {
      h = parse_head(sv);
    } catch (const std::invalid_argument& e) {
      throw py::value_error(e.what());
    }
    return py::make_tuple(py::str(h.a), py::str(h.b), py::str(h.c), headers_dict(h.headers));
  });

  py::class_<TxOp>(m, "TxOp")
      .def(py::init([](bool is_delete, std::string key, std::string value, std::optional<std::string> etag,
                       bool first_write, int64_t ttl_ms) {
             TxOp op;
             op.is_delete = is_delete;
             op.key = std::move(key);
             op.value = std::move(value);
             op.etag = std::move(etag);
             op.first_write = first_write;
             op.ttl_ms = ttl_ms;
             return op;
           }),
           py::arg("is_delete"), py::arg("key"), py::arg("value") = "", py::arg("etag") = std::nullopt,
           py::arg("first_write") = false, py::arg("ttl_ms") = 0)
      .def_readonly("is_delete", &TxOp::is_delete)
      .def_readonly("key", &TxOp::key)
      .def_readonly("value", &TxOp::value)
      .def_readonly("ttl_ms", &TxOp::ttl_ms);

  py::class_<DocStore>(m, "DocStore")
      .def(py::init<const std::string&, int, size_t>(), py::arg("path") = "", py::arg("fsync_mode") = 0,
           py::arg("index_threshold") = 256)
      .def("set", &DocStore::set, py::arg("key"), py::arg("value"), py::arg("etag") = std::nullopt,
           py::arg("first_write") = false, py::arg("ttl_ms") = 0, py::call_guard<py::gil_scoped_release>())
      .def("get", &DocStore::get, py::arg("key"))
      .def("delete", &DocStore::del, py::arg("key"), py::arg("etag") = std::nullopt)
      .def("transact", &DocStore::transact, py::arg("ops"), py::call_guard<py::gil_scoped_release>())
      .def("query", &DocStore::query, py::arg("query"), py::arg("prefix") = "",
           py::call_guard<py::gil_scoped_release>())
      .def("keys", &DocStore::keys, py::arg("prefix") = "", py::arg("limit") = 0)
      .def("encode_columns",
           [](DocStore& s, const std::string& prefix, const std::vector<std::string>& paths) {
             DocStore::Encoded e;
             {
               py::gil_scoped_release r;
               e = s.encode_columns(prefix, paths);
             }
             py::list cols;
             for (auto& c : e.cols) {
               py::array_t<int32_t> ids((py::ssize_t)c.ids.size());
               std::memcpy(ids.mutable_data(), c.ids.data(), c.ids.size() * sizeof(int32_t));
               cols.append(py::make_tuple(py::cast(c.values), ids));
             }
             py::array_t<int64_t> seqs((py::ssize_t)e.seqs.size());
             std::memcpy(seqs.mutable_data(), e.seqs.data(), e.seqs.size() * sizeof(int64_t));
             py::array_t<int64_t> offs((py::ssize_t)e.key_off.size());
             std::memcpy(offs.mutable_data(), e.key_off.data(), e.key_off.size() * sizeof(int64_t));
             // keys stay one bytes blob + offsets: no per-document Python string objects
             return py::make_tuple(py::make_tuple(py::bytes(e.key_blob), offs), seqs, cols);
           },
           py::arg("prefix"), py::arg("paths"))
      .def("mirror_enable", &DocStore::mirror_enable, py::arg("paths"), py::call_guard<py::gil_scoped_release>())
      .def("mirror_delta",
           [](DocStore& s, uint64_t gen, size_t from, size_t kill_from, const std::vector<size_t>& dict_sizes) {
             MirrorDelta d;
             {
               py::gil_scoped_release r;
               d = s.mirror_delta(gen, from, kill_from, dict_sizes);
             }
             auto arr = [](const auto& v) {
               using T = typename std::decay_t<decltype(v)>::value_type;
               py::array_t<T> a((py::ssize_t)v.size());
               if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
               return a;
             };
             py::list cols;
             for (size_t c = 0; c < d.paths.size(); ++c)
               cols.append(py::make_tuple(d.paths[c], d.dict_from[c], py::cast(d.new_values[c]), arr(d.ids[c])));
             py::dict out;
             out["gen"] = d.gen;
             out["on"] = d.on;
             out["disabled"] = d.disabled;
             out["full"] = d.full;
             out["n"] = d.n;
             out["from"] = d.from;
             out["kill_cursor"] = d.kill_cursor;
             out["kills"] = arr(d.kills);
             out["seqs"] = arr(d.seqs);
             out["live"] = arr(d.live);
             out["columns"] = cols;
             return out;
           },
           py::arg("gen"), py::arg("from_row"), py::arg("kill_from"), py::arg("dict_sizes"))
      .def("mirror_results",
           [](DocStore& s, py::array_t<int32_t, py::array::c_style | py::array::forcecast> rows,
              const std::string& prefix, const std::string& token) {
             size_t skipped = 0;
             std::string out;
             const int32_t* p = rows.data();
             size_t n = (size_t)rows.size();
             {
               py::gil_scoped_release r;
               out = s.mirror_results(p, n, prefix, token, &skipped);
             }
             return py::make_tuple(py::bytes(out), skipped);
           },
           py::arg("rows"), py::arg("prefix") = "", py::arg("token") = "")
      .def("mirror_stats", &DocStore::mirror_stats)
      .def("set_throughput", &DocStore::set_throughput, py::arg("ru_per_s"))
      .def("charge", &DocStore::charge, py::arg("ru"))
      .def("throughput_stats", &DocStore::throughput_stats)
      .def_static("read_ru", &DocStore::read_ru)
      .def_static("write_ru", &DocStore::write_ru)
      .def_static("query_ru", &DocStore::query_ru)
      .def("size", &DocStore::size)
      .def("__len__", &DocStore::size)
      .def("compact", &DocStore::compact)
      .def("sync", &DocStore::sync)
      .def("stats", &DocStore::stats)
      .def("indexed_paths", &DocStore::indexed_paths);

  py::class_<QueueOptions>(m, "QueueOptions")
      .def(py::init([](int64_t lock_ms, uint32_t max_delivery, int64_t default_ttl_ms, bool dead_letter_on_expiry) {
             QueueOptions o;
             o.lock_ms = lock_ms;
             o.max_delivery = max_delivery;
             o.default_ttl_ms = default_ttl_ms;
             o.dead_letter_on_expiry = dead_letter_on_expiry;
             return o;
           }),
           py::arg("lock_ms") = 60000, py::arg("max_delivery") = 10, py::arg("default_ttl_ms") = 0,
           py::arg("dead_letter_on_expiry") = false)
      .def_readwrite("lock_ms", &QueueOptions::lock_ms)
      .def_readwrite("max_delivery", &QueueOptions::max_delivery)
      .def_readwrite("default_ttl_ms", &QueueOptions::default_ttl_ms)
      .def_readwrite("dead_letter_on_expiry", &QueueOptions::dead_letter_on_expiry);

  py::class_<Received>(m, "Received")
      .def_readonly("lock_token", &Received::lock_token)
      .def_readonly("seq", &Received::seq)
      .def_readonly("id", &Received::id)
      .def_property_readonly("body", [](const Received& r) { return py::bytes(r.body); })
      .def_readonly("content_type", &Received::content_type)
      .def_readonly("props", &Received::props)
      .def_readonly("delivery_count", &Received::delivery_count)
      .def_readonly("enqueued_ms", &Received::enqueued_wall);

  py::class_<Broker>(m, "Broker")
      .def(py::init<const std::string&, int>(), py::arg("path") = "", py::arg("fsync_mode") = 0)
      .def("create_queue", &Broker::create_queue, py::arg("name"), py::arg("options") = QueueOptions())
      .def("create_topic", &Broker::create_topic)
      .def("create_subscription", &Broker::create_subscription, py::arg("topic"), py::arg("subscription"),
           py::arg("options") = QueueOptions())
      .def("delete_entity", &Broker::delete_entity)
      .def("subscriptions", &Broker::subscriptions)
      .def("entities", &Broker::entities)
      .def("publish",
           [](Broker& b, const std::string& topic, py::bytes body, const std::string& ctype, const std::string& props,
              const std::string& id, int64_t ttl_ms, int64_t delay_ms) {
             std::string s = body;
             py::gil_scoped_release r;
             return b.publish(topic, s, ctype, props, id, ttl_ms, delay_ms);
           },
           py::arg("topic"), py::arg("body"), py::arg("content_type") = "application/json", py::arg("props") = "{}",
           py::arg("id") = "", py::arg("ttl_ms") = 0, py::arg("delay_ms") = 0)
      .def("send",
           [](Broker& b, const std::string& q, py::bytes body, const std::string& ctype, const std::string& props,
              const std::string& id, int64_t ttl_ms, int64_t delay_ms) {
             std::string s = body;
             py::gil_scoped_release r;
             return b.send(q, s, ctype, props, id, ttl_ms, delay_ms);
           },
           py::arg("queue"), py::arg("body"), py::arg("content_type") = "application/json", py::arg("props") = "{}",
           py::arg("id") = "", py::arg("ttl_ms") = 0, py::arg("delay_ms") = 0)
      .def("receive", &Broker::receive, py::arg("path"), py::arg("max_messages") = 1, py::arg("lock_ms") = 0)
      .def("complete", &Broker::complete)
      .def("abandon", &Broker::abandon, py::arg("path"), py::arg("token"), py::arg("delay_ms") = 0)
      .def("dead_letter", &Broker::dead_letter, py::arg("path"), py::arg("token"), py::arg("reason") = "")
      .def("renew", &Broker::renew, py::arg("path"), py::arg("token"), py::arg("lock_ms") = 0)
      .def("drain_dead_letters",
           [](Broker& b, const std::string& path, size_t max) {
             py::list out;
             for (auto& [seq, id, body, reason, dc] : b.drain_dead_letters(path, max))
               out.append(py::make_tuple(seq, id, py::bytes(body), reason, dc));
             return out;
           },
           py::arg("path"), py::arg("max") = 100)
      .def("counts",
           [](Broker& b, const std::string& path) {
             auto [a, s, l, d, e, c, r] = b.counts(path);
             py::dict out;
             out["active"] = a;
             out["scheduled"] = s;
             out["locked"] = l;
             out["dead_letter"] = d;
             out["enqueued"] = e;
             out["completed"] = c;
             out["received"] = r;
             return out;
           })
      .def("purge", &Broker::purge)
      .def("total_published", &Broker::total_published);

  // Native HTTP front of the backing-services process (backingfront.hpp): serves the hot
  // document / message routes on its own thread against the engines attached here and
  // forwards everything else to the Python server on `fallback_uds`.
  py::class_<BackingFront>(m, "BackingFront")
      .def(py::init<const std::string&, int, const std::string&, int>(), py::arg("host"), py::arg("port"),
           py::arg("fallback_uds"), py::arg("threads") = 1)
      .def("port", &BackingFront::port)
      .def("threads", &BackingFront::threads)
      .def("attach_store",
           [](BackingFront& f, const std::string& a, const std::string& d, const std::string& c, DocStore& s) {
             f.attach_store(a, d, c, &s);
           },
           py::keep_alive<1, 5>())
      .def("attach_broker", [](BackingFront& f, const std::string& ns, Broker& b) { f.attach_broker(ns, &b); },
           py::keep_alive<1, 3>())
      .def("set_policy", &BackingFront::set_policy, py::arg("mode"), py::arg("keys"), py::arg("grants"))
      .def("notify", &BackingFront::notify)
      .def("stats", &BackingFront::stats)
      .def("stop", &BackingFront::stop, py::call_guard<py::gil_scoped_release>());

  // Native HTTP host of an app process (apphost.hpp): its epoll thread owns the listeners and
  // the client pools; Python hands it responses and outbound requests in batches (submit()),
  // collects parsed requests and responses with drain() and waits on event_fd().
  py::class_<apphost::AppHost>(m, "AppHost")
      .def(py::init<>())
      .def("start", &apphost::AppHost::start)
      .def("stop", &apphost::AppHost::stop, py::call_guard<py::gil_scoped_release>())
      .def("event_fd", &apphost::AppHost::event_fd)
      .def("listen", &apphost::AppHost::listen, py::arg("server"), py::arg("endpoint"), py::arg("cert") = "",
           py::arg("key") = "", py::call_guard<py::gil_scoped_release>())
      .def("close_server", &apphost::AppHost::close_server)
      .def("close_connections", &apphost::AppHost::close_connections)
      .def("pending_replies", &apphost::AppHost::pending_replies)
      // ops: [(0, token, status, headers, body) | (1, id, endpoint, method, target, headers, body, timeout) |
      //       (2, id, endpoint, "", grpc_path, metadata, message, timeout)]
      .def("submit",
           [](apphost::AppHost& h, py::list ops) {
             std::vector<apphost::AppHost::Op> v;
             v.reserve(ops.size());
             for (auto item : ops) {
               auto t = item.cast<py::tuple>();
               apphost::AppHost::Op op;
               int kind = t[0].cast<int>();
               op.is_request = kind == 1 || kind == 2;
               op.is_grpc = kind == 2;
               op.id = t[1].cast<uint64_t>();
               if (!op.is_request) {
                 op.status = t[2].cast<int>();
                 op.headers = header_list(t[3]);
                 op.body = bytes_of(t[4]);
               } else {
                 op.endpoint = t[2].cast<std::string>();
                 op.method = t[3].cast<std::string>();
                 op.target = t[4].cast<std::string>();
                 op.headers = header_list(t[5]);
                 op.body = bytes_of(t[6]);
                 op.timeout_s = t[7].cast<double>();
               }
               v.push_back(std::move(op));
             }
             h.submit(std::move(v));
           })
      // [(0, token, server, method, target, http10, headers, body) | (1, id, status, headers, body) |
      //  (2, id, errno, message)]
      .def("drain_times", [](apphost::AppHost& h) {
        // same as drain() plus each event's queue time (monotonic seconds) as the last element
        auto evs = h.drain();
        py::list out;
        for (auto& e : evs) {
          if (e.kind == apphost::Event::REQUEST) {
            out.append(py::make_tuple(0, e.id, e.server, py::str(e.msg.method), py::str(e.msg.target),
                                      e.msg.http10, headers_dict(e.msg.headers), py::bytes(e.msg.body), e.t));
          } else if (e.kind == apphost::Event::RESPONSE) {
            out.append(py::make_tuple(1, e.id, e.msg.status, headers_dict(e.msg.headers), py::bytes(e.msg.body), e.t));
          } else {
            out.append(py::make_tuple(2, e.id, e.err, py::str(std::strerror(e.err)), e.t));
          }
        }
        return out;
      })
      .def("drain", [](apphost::AppHost& h) {
        auto evs = h.drain();
        py::list out;
        for (auto& e : evs) {
          if (e.kind == apphost::Event::REQUEST) {
            out.append(py::make_tuple(0, e.id, e.server, py::str(e.msg.method), py::str(e.msg.target),
                                      e.msg.http10, headers_dict(e.msg.headers), py::bytes(e.msg.body)));
          } else if (e.kind == apphost::Event::RESPONSE) {
            out.append(py::make_tuple(1, e.id, e.msg.status, headers_dict(e.msg.headers), py::bytes(e.msg.body)));
          } else {
            out.append(py::make_tuple(2, e.id, e.err, py::str(std::strerror(e.err))));
          }
        }
        return out;
      });
}
