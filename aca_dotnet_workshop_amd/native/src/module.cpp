// Python bindings for the native state-store and broker engines (`_ttnative`).
#include <unistd.h>

#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include "apphost.hpp"
#include "daprpb.hpp"
#include "backingfront.hpp"
#include "broker.hpp"
#include "cpuscan.hpp"
#include "docstore.hpp"
#include "dutycycle.hpp"
#include "httpparse.hpp"
#include "taskcodec.hpp"
#include "sweepcodec.hpp"
#include "pcsample.hpp"
#include "formcodec.hpp"
#include "strrank.hpp"

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

// ---- raw CPython conversions for the app host's per-request hand-offs (submit / drain run for
// every request and response of a service process; pybind11's generic casters cost several
// microseconds per operation there).
static std::string_view utf8_view(PyObject* o) {
  Py_ssize_t n;
  const char* p = PyUnicode_AsUTF8AndSize(o, &n);
  if (p == nullptr) throw py::error_already_set();
  return std::string_view(p, (size_t)n);
}

static std::string str_of(PyObject* o) {  // like f"{o}"
  if (PyUnicode_Check(o)) return std::string(utf8_view(o));
  py::object s = py::reinterpret_steal<py::object>(PyObject_Str(o));
  if (!s) throw py::error_already_set();
  return std::string(utf8_view(s.ptr()));
}

static std::string_view need_str(PyObject* o, const char* what) {
  if (!PyUnicode_Check(o)) throw py::type_error(std::string(what) + " must be a str");
  return utf8_view(o);
}

static long long need_int(PyObject* o, const char* what) {
  long long v = PyLong_AsLongLong(o);
  if (v == -1 && PyErr_Occurred()) {
    PyErr_Clear();
    throw py::type_error(std::string(what) + " must be an int");
  }
  return v;
}

static py::object seq_fast(PyObject* o, const char* what) {
  py::object f = py::reinterpret_steal<py::object>(PySequence_Fast(o, what));
  if (!f) throw py::error_already_set();
  return f;
}

static ev::HeaderList header_list_fast(PyObject* seq) {
  py::object f = seq_fast(seq, "headers must be a sequence of (name, value)");
  Py_ssize_t n = PySequence_Fast_GET_SIZE(f.ptr());
  PyObject** items = PySequence_Fast_ITEMS(f.ptr());
  ev::HeaderList out;
  out.reserve((size_t)n);
  for (Py_ssize_t i = 0; i < n; ++i) {
    py::object kv = seq_fast(items[i], "a header must be a (name, value) pair");
    if (PySequence_Fast_GET_SIZE(kv.ptr()) != 2) throw py::value_error("a header must be a (name, value) pair");
    PyObject** p = PySequence_Fast_ITEMS(kv.ptr());
    std::string k(need_str(p[0], "header name"));
    for (auto& ch : k) ch = (char)std::tolower((unsigned char)ch);
    out.emplace_back(std::move(k), str_of(p[1]));
  }
  return out;
}

static std::string body_of(PyObject* o) {
  char* p;
  Py_ssize_t n;
  if (PyBytes_AsStringAndSize(o, &p, &n) != 0) throw py::error_already_set();
  return std::string(p, (size_t)n);
}

// Steals `v`; throws if it is null (a failed allocation / conversion).
static void set_item(PyObject* tup, Py_ssize_t i, PyObject* v) {
  if (v == nullptr) throw py::error_already_set();
  PyTuple_SET_ITEM(tup, i, v);
}

static PyObject* new_str(const std::string& s) { return PyUnicode_DecodeUTF8(s.data(), (Py_ssize_t)s.size(), "replace"); }

// headers_dict() without pybind11: lower-cased names, repeats joined by ", ", set-cookie a list.
static PyObject* headers_dict_fast(const ev::HeaderList& headers) {
  py::object d = py::reinterpret_steal<py::object>(PyDict_New());
  if (!d) throw py::error_already_set();
  for (auto& [k, v] : headers) {
    py::object key = py::reinterpret_steal<py::object>(new_str(k));
    py::object val = py::reinterpret_steal<py::object>(new_str(v));
    if (!key || !val) throw py::error_already_set();
    PyObject* prev = PyDict_GetItemWithError(d.ptr(), key.ptr());  // borrowed
    if (prev == nullptr && PyErr_Occurred()) throw py::error_already_set();
    if (prev == nullptr) {
      if (PyDict_SetItem(d.ptr(), key.ptr(), val.ptr()) != 0) throw py::error_already_set();
    } else if (k == "set-cookie") {
      if (PyList_Check(prev)) {
        if (PyList_Append(prev, val.ptr()) != 0) throw py::error_already_set();
      } else {
        py::object l = py::reinterpret_steal<py::object>(PyList_New(2));
        if (!l) throw py::error_already_set();
        Py_INCREF(prev);
        PyList_SET_ITEM(l.ptr(), 0, prev);
        PyList_SET_ITEM(l.ptr(), 1, val.release().ptr());
        if (PyDict_SetItem(d.ptr(), key.ptr(), l.ptr()) != 0) throw py::error_already_set();
      }
    } else {
      std::string joined = str_of(prev) + ", " + v;
      py::object j = py::reinterpret_steal<py::object>(new_str(joined));
      if (!j || PyDict_SetItem(d.ptr(), key.ptr(), j.ptr()) != 0) throw py::error_already_set();
    }
  }
  return d.release().ptr();
}

static py::list events_to_py(std::vector<apphost::Event>& evs, bool with_times) {
  // the finished log lines of the batch (native routes' records on the JSON sink's fast path)
  // go up as ONE event per run of consecutive lines of one (level, logger): (4, level, logger
  // name, the lines joined) -- two lines per created task otherwise cost a tuple, a call and a
  // sink lock each in Python.  A run keeps its place among the other events, so the log's order
  // is the order the I/O thread produced it in.
  struct Item {
    long batch = -1;  // >= 0: a run of lines; else the event `ev`
    size_t ev = 0;
  };
  std::vector<Item> items;
  items.reserve(evs.size());
  std::vector<std::pair<std::pair<int, std::string>, std::string>> batches;
  for (size_t i = 0; i < evs.size(); ++i) {
    auto& e = evs[i];
    if (e.kind != apphost::Event::LOG || e.line.empty() || with_times) {
      items.push_back({-1, i});
      continue;
    }
    auto key = std::make_pair(e.err, e.msg.method);
    if (!items.empty() && items.back().batch >= 0 && batches[(size_t)items.back().batch].first == key) {
      batches[(size_t)items.back().batch].second += e.line;
      continue;
    }
    batches.emplace_back(key, e.line);
    items.push_back({(long)batches.size() - 1, 0});
  }
  py::list out(items.size());
  for (size_t ki = 0; ki < items.size(); ++ki) {
    if (items[ki].batch < 0) continue;
    auto& b = batches[(size_t)items[ki].batch];
    py::object t = py::reinterpret_steal<py::object>(PyTuple_New(4));
    if (!t) throw py::error_already_set();
    set_item(t.ptr(), 0, PyLong_FromLong(4));
    set_item(t.ptr(), 1, PyLong_FromLong(b.first.first));
    set_item(t.ptr(), 2, new_str(b.first.second));
    set_item(t.ptr(), 3, new_str(b.second));
    PyList_SET_ITEM(out.ptr(), (Py_ssize_t)ki, t.release().ptr());
  }
  for (size_t ki = 0; ki < items.size(); ++ki) {
    if (items[ki].batch >= 0) continue;
    auto& e = evs[items[ki].ev];
    py::object t;
    if (e.kind == apphost::Event::REQUEST) {
      t = py::reinterpret_steal<py::object>(PyTuple_New(with_times ? 9 : 8));
      if (!t) throw py::error_already_set();
      set_item(t.ptr(), 0, PyLong_FromLong(0));
      set_item(t.ptr(), 1, PyLong_FromUnsignedLongLong(e.id));
      set_item(t.ptr(), 2, PyLong_FromLong(e.server));
      set_item(t.ptr(), 3, new_str(e.msg.method));
      set_item(t.ptr(), 4, new_str(e.msg.target));
      set_item(t.ptr(), 5, PyBool_FromLong(e.msg.http10));
      set_item(t.ptr(), 6, headers_dict_fast(e.msg.headers));
      set_item(t.ptr(), 7, PyBytes_FromStringAndSize(e.msg.body.data(), (Py_ssize_t)e.msg.body.size()));
      if (with_times) set_item(t.ptr(), 8, PyFloat_FromDouble(e.t));
    } else if (e.kind == apphost::Event::RESPONSE) {
      t = py::reinterpret_steal<py::object>(PyTuple_New(with_times ? 6 : 5));
      if (!t) throw py::error_already_set();
      set_item(t.ptr(), 0, PyLong_FromLong(1));
      set_item(t.ptr(), 1, PyLong_FromUnsignedLongLong(e.id));
      set_item(t.ptr(), 2, PyLong_FromLong(e.msg.status));
      set_item(t.ptr(), 3, headers_dict_fast(e.msg.headers));
      set_item(t.ptr(), 4, PyBytes_FromStringAndSize(e.msg.body.data(), (Py_ssize_t)e.msg.body.size()));
      if (with_times) set_item(t.ptr(), 5, PyFloat_FromDouble(e.t));
    } else if (e.kind == apphost::Event::LOG) {
      // (3, level, logger name, message, trace id, span id, finished line or "")
      t = py::reinterpret_steal<py::object>(PyTuple_New(with_times ? 8 : 7));
      if (!t) throw py::error_already_set();
      set_item(t.ptr(), 0, PyLong_FromLong(3));
      set_item(t.ptr(), 1, PyLong_FromLong(e.err));
      set_item(t.ptr(), 2, new_str(e.msg.method));
      set_item(t.ptr(), 3, new_str(e.msg.body));
      set_item(t.ptr(), 4, new_str(e.msg.target));
      set_item(t.ptr(), 5, new_str(e.msg.reason));
      set_item(t.ptr(), 6, new_str(e.line));
      if (with_times) set_item(t.ptr(), 7, PyFloat_FromDouble(e.t));
    } else {
      if (with_times) t = py::make_tuple(2, e.id, e.err, py::str(std::strerror(e.err)), e.t);
      else t = py::make_tuple(2, e.id, e.err, py::str(std::strerror(e.err)));
    }
    PyList_SET_ITEM(out.ptr(), (Py_ssize_t)ki, t.release().ptr());
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
  // TT_PC_SAMPLE for a Python process that hosts native engines (the backing services): the
  // process's CPU time sampled by program counter, the interpreter's share included
  // (pcsample.hpp); dump at exit
  // Growth points of the store's sharded key map: insert n GUID-like keys (as the task ids are)
  // and return, per insert at which any shard grew, [insert index, shards grown].
  m.def("sharded_map_growth", [](size_t n) {
    tt::ShardedMap<int32_t> map;
    constexpr size_t S = tt::ShardedMap<int32_t>::shards();
    std::vector<size_t> bkt(S);
    for (size_t s = 0; s < S; ++s) bkt[s] = map.bucket_count(s);
    std::vector<std::pair<size_t, size_t>> out;
    uint64_t x = 0x9e3779b97f4a7c15ull;
    char key[37];
    for (size_t i = 0; i < n; ++i) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      uint64_t y = x * 0x2545f4914f6cdd1dull;
      std::snprintf(key, sizeof key, "%08x-%04x-4%03x-a%03x-%012llx", (unsigned)(x >> 32), (unsigned)(x >> 16) & 0xffff,
                    (unsigned)x & 0xfff, (unsigned)(y >> 52), (unsigned long long)(y & 0xffffffffffffull));
      map[key] = (int32_t)i;
      size_t grown = 0;
      for (size_t s = 0; s < S; ++s)
        if (map.bucket_count(s) != bkt[s]) bkt[s] = map.bucket_count(s), ++grown;
      if (grown) out.emplace_back(i, grown);
    }
    return out;
  }, py::call_guard<py::gil_scoped_release>());
  m.def("pc_sample_start", [] { tt::pcsample::start(); });
  m.def("pc_sample_dump", [](const std::string& who) { tt::pcsample::dump(who.c_str()); },
        py::call_guard<py::gil_scoped_release>());
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
  // CPU time (ns) of each thread whose /proc/<pid>/task/<tid>/schedstat is open on the given
  // descriptor (-1: unreadable, e.g. the thread exited): the watchdog CPU throttle of
  // platform/limits.py reads every replica thread each tick in one call, at nanosecond
  // resolution (utime/stime in /proc/<pid>/stat count 10 ms clock ticks).
  m.def("schedstat_ns", [](const std::vector<int>& fds) {
    std::vector<long long> out(fds.size(), -1);
    {
      py::gil_scoped_release r;
      char buf[128];
      for (size_t i = 0; i < fds.size(); ++i) {
        ssize_t n = ::pread(fds[i], buf, sizeof buf - 1, 0);
        if (n <= 0) continue;
        buf[n] = 0;
        char* end = nullptr;
        long long v = std::strtoll(buf, &end, 10);
        if (end != buf) out[i] = v;
      }
    }
    return out;
  });
  // bulkset body -> the stored text of each item's value (backingfront.hpp scan_bulk_values), or None.
  m.def("bulk_values", [](py::bytes body) -> py::object {
    std::string b = body;
    std::vector<std::string> vals;
    if (!scan_bulk_values(b, vals)) return py::none();
    py::list l(vals.size());
    for (size_t i = 0; i < vals.size(); ++i) l[i] = py::str(vals[i]);
    return l;
  });

  // transaction body -> the stored text of each op's value (backingfront.hpp scan_tx_values), or None.
  m.def("tx_values", [](py::bytes body) -> py::object {
    std::string b = body;
    std::vector<std::string> vals;
    if (!scan_tx_values(b, vals)) return py::none();
    py::list l(vals.size());
    for (size_t i = 0; i < vals.size(); ++i) l[i] = py::str(vals[i]);
    return l;
  });

  // The watchdog CPU duty cycle on a native thread (dutycycle.hpp; platform/limits.py).
  py::class_<DutyCycle>(m, "DutyCycle")
      .def(py::init<double>(), py::arg("period_s"))
      .def("add", &DutyCycle::add, py::arg("name"), py::arg("pid"), py::arg("cpu"),
           py::call_guard<py::gil_scoped_release>())
      .def("remove", &DutyCycle::remove, py::arg("name"), py::call_guard<py::gil_scoped_release>())
      .def("start", &DutyCycle::start)
      .def("stop", &DutyCycle::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("period_s", &DutyCycle::period_s)
      .def("stats", [](DutyCycle& d) {
        std::map<std::string, DutyCycle::Stats> st;
        {
          py::gil_scoped_release r;
          st = d.stats();
        }
        py::dict out;
        for (auto& kv : st) {
          py::dict x;
          x["throttled_periods"] = kv.second.throttled_periods;
          x["cpu_seconds"] = kv.second.cpu_seconds;
          x["stopped_seconds"] = kv.second.stopped_seconds;
          x["stopped"] = kv.second.stopped;
          out[py::str(kv.first)] = x;
        }
        return out;
      });
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

  // TaskAddModel body -> (id, taskName, taskAssignedTo, TaskModel JSON, state-save body), or
  // None when the general (pydantic) binder must decide (taskcodec.hpp).
  m.def("task_create", [](py::bytes body) -> py::object {
    static taskcodec::Entropy rng;  // called with the GIL held
    static taskcodec::Created c;
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    if (!taskcodec::create(std::string_view(p, (size_t)n), rng, c)) return py::none();
    return py::make_tuple(py::str(c.id), py::str(c.name), py::str(c.assigned_to),
                          py::bytes(c.task_json), py::bytes(c.state_body));
  });

  // CloudEvents envelope -> (data JSON, datacontenttype, attributes dict), or None (taskcodec.hpp).
  m.def("cloudevent_unwrap", [](py::bytes body) -> py::object {
    static taskcodec::Unwrapped u;
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    if (!taskcodec::unwrap_cloudevent(std::string_view(p, (size_t)n), u)) return py::none();
    py::dict attrs;
    for (const auto& kv : u.attrs) {
      const tt::Value& v = *kv.second;
      py::object o;
      if (v.t == tt::Value::String) o = py::str(v.s);
      else if (v.t == tt::Value::Bool) o = py::bool_(v.b);
      else if (v.t == tt::Value::Null) o = py::none();
      else o = py::module_::import("json").attr("loads")(py::str(tt::dump(v)));
      attrs[py::str(kv.first)] = o;
    }
    return py::make_tuple(py::bytes(u.data), py::str(u.content_type), attrs);
  });

  // markoverdue body -> (ids, bulk-save body) or None (taskcodec.hpp mark_overdue).
  m.def("tasks_mark_overdue", [](py::bytes body) -> py::object {
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    std::vector<std::string> ids;
    std::string bulk;
    if (!taskcodec::mark_overdue(std::string_view(p, (size_t)n), ids, bulk)) return py::none();
    py::list l(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) l[i] = py::str(ids[i]);
    return py::make_tuple(l, py::bytes(bulk));
  });

  // dapr.proto.runtime.v1 messages of the gRPC SDK's hot calls (daprpb.hpp), shared with the app
  // host's native routes: the same bytes from both.
  auto view = [](const py::bytes& b) {
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(b.ptr(), &p, &n) != 0) throw py::error_already_set();
    return std::string_view(p, (size_t)n);
  };
  // the state API's save body -> SaveStateRequest, or None
  m.def("dapr_pb_save_state_bulk", [view](const std::string& store, py::bytes body) -> py::object {
    std::string out;
    if (!tt::daprpb::save_state_bulk(store, view(body), out)) return py::none();
    return py::bytes(out);
  });
  m.def("dapr_pb_get_bulk_state", [](const std::string& store, const std::vector<std::string>& keys, int parallelism) {
    return py::bytes(tt::daprpb::get_bulk_state(store, keys, parallelism));
  });
  // GetBulkStateResponse -> the bulk-get API's JSON ([{"key","data","etag"} | {"key"}]), or None
  m.def("dapr_pb_bulk_state_json", [view](py::bytes msg) -> py::object {
    std::string out;
    if (!tt::daprpb::bulk_state_response_json(view(msg), out)) return py::none();
    return py::bytes(out);
  });
  // the query API's JSON -> QueryStateResponse (the sidecar's one-pass encoder), or None
  m.def("dapr_pb_query_from_json", [view](py::bytes body) -> py::object {
    std::string out;
    if (!tt::daprpb::query_response_pb(view(body), out)) return py::none();
    return py::bytes(out);
  });
  // the sweep's one-pass pb hops (sweepcodec.hpp), or None where the caller runs the chain
  m.def("tasks_from_query_pb", [view](py::bytes msg, bool by_created, bool descending) -> py::object {
    std::string out;
    size_t count = 0;
    bool more = false;
    if (!taskcodec::query_pb_tasks(view(msg), out, count, by_created, &more, descending)) return py::none();
    return py::make_tuple(count, py::bytes(out), more);
  });
  m.def("tasks_conditional_mark_pb", [view](py::bytes msg, const std::string& store) -> py::object {
    std::string save;
    std::vector<std::string> ids;
    size_t skipped = 0;
    if (!taskcodec::conditional_mark_pb(view(msg), store, save, ids, skipped)) return py::none();
    return py::make_tuple(py::bytes(save), ids, skipped);
  });
  m.def("tasks_mark_overdue_ids", [view](py::bytes body) -> py::object {
    std::vector<std::string> ids;
    if (!taskcodec::mark_overdue_ids(view(body), ids)) return py::none();
    return py::cast(ids);
  });
  // QueryStateResponse -> the query API's JSON ({"results":[..],"token"}), or None
  m.def("dapr_pb_query_json", [view](py::bytes msg) -> py::object {
    std::string out;
    if (!tt::daprpb::query_response_json(view(msg), out)) return py::none();
    return py::bytes(out);
  });

  // The API's read-modify-writes (taskcodec.hpp edit_task / bind_update / task_json): one
  // native pass each, shared with the app host's native routes.
  // PUT api/tasks/{id} body -> (name, assigned_to, due) or None (the general binder decides)
  m.def("task_update_bind", [view](py::bytes body) -> py::object {
    taskcodec::Update u;
    if (!taskcodec::bind_update(view(body), u)) return py::none();
    return py::make_tuple(py::str(u.name), py::str(u.assigned_to), py::str(u.due));
  });
  // stored task + the edit -> (document to write back, id, stored assignee) or None.  `update`:
  // (name, assigned_to, due) from task_update_bind, or None (markcomplete: `complete`)
  m.def("task_edit", [view](py::bytes stored, bool complete, py::object update) -> py::object {
    taskcodec::Update u;
    const taskcodec::Update* up = nullptr;
    if (!update.is_none()) {
      auto t = update.cast<py::tuple>();
      u.name = t[0].cast<std::string>();
      u.assigned_to = t[1].cast<std::string>();
      u.due = t[2].cast<std::string>();
      up = &u;
    }
    std::string out, id, old;
    if (!taskcodec::edit_task(view(stored), up, complete, out, id, old)) return py::none();
    return py::make_tuple(py::bytes(out), py::str(id), py::str(old));
  });
  // stored task -> its TaskModel JSON (GET api/tasks/{id}) or None
  m.def("task_json", [view](py::bytes stored) -> py::object {
    std::string out;
    if (!taskcodec::task_json(view(stored), out)) return py::none();
    return py::bytes(out);
  });
  // (a, b) -> True / False (ASCII case-insensitive equality), None when either is not ASCII
  m.def("ascii_ieq", [](const std::string& a, const std::string& b) -> py::object {
    int r = taskcodec::ascii_ieq(a, b);
    if (r < 0) return py::none();
    return py::bool_(r == 1);
  });

  // bulk-get answer for a markoverdue page -> (ids marked, conditional bulk-save body, skipped)
  // or None (taskcodec.hpp conditional_mark).
  m.def("tasks_conditional_mark", [](py::bytes got) -> py::object {
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(got.ptr(), &p, &n) != 0) throw py::error_already_set();
    std::vector<std::string> ids;
    std::string bulk;
    size_t skipped = 0;
    if (!taskcodec::conditional_mark(std::string_view(p, (size_t)n), bulk, ids, skipped)) return py::none();
    py::list l(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) l[i] = py::str(ids[i]);
    return py::make_tuple(l, py::bytes(bulk), skipped);
  });

  // overdue page + run date (YYYY-MM-DD) -> (retrieved, kept, TaskModel JSON array) or None.
  m.def("tasks_overdue_filter", [](py::bytes body, const std::string& run_day) -> py::object {
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    size_t retrieved = 0, kept = 0;
    std::string out;
    if (!taskcodec::overdue_filter(std::string_view(p, (size_t)n), run_day, retrieved, kept, out)) return py::none();
    return py::make_tuple(retrieved, kept, py::bytes(out));
  });

  // overdue page + run date + chunk size -> (retrieved, kept, [TaskModel JSON arrays of at most
  // `chunk` tasks each]) or None: the filter and the processor's markoverdue chunks in one pass.
  m.def("tasks_overdue_filter_chunks", [](py::bytes body, const std::string& run_day, size_t chunk) -> py::object {
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    if (chunk == 0) return py::none();
    size_t retrieved = 0, kept = 0;
    std::string out;
    std::vector<size_t> starts;
    if (!taskcodec::overdue_filter(std::string_view(p, (size_t)n), run_day, retrieved, kept, out, &starts))
      return py::none();
    py::list parts;
    const size_t body_end = out.size() - 1;  // the closing ']'
    for (size_t a = 0; a < starts.size(); a += chunk) {
      const size_t b = std::min(starts.size(), a + chunk);
      const size_t from = starts[a], to = b < starts.size() ? starts[b] - 1 : body_end;  // drop the ','
      std::string part;
      part.reserve(to - from + 2);
      part += '[';
      part.append(out, from, to - from);
      part += ']';
      parts.append(py::bytes(part));
    }
    return py::make_tuple(retrieved, kept, parts);
  });

  // The frontend's Create post (formcodec.hpp): None = the page decides; (True, TaskAddModel JSON)
  // = send it to api/tasks; (False, b"") = the antiforgery token is invalid (400).
  m.def("frontend_create_form", [](py::bytes body, py::bytes cookie, py::bytes key) -> py::object {
    char *pb, *pc, *pk;
    Py_ssize_t nb, nc, nk;
    if (PyBytes_AsStringAndSize(body.ptr(), &pb, &nb) != 0 || PyBytes_AsStringAndSize(cookie.ptr(), &pc, &nc) != 0 ||
        PyBytes_AsStringAndSize(key.ptr(), &pk, &nk) != 0)
      throw py::error_already_set();
    std::string json;
    auto v = formcodec::create_task(std::string_view(pb, (size_t)nb), std::string_view(pc, (size_t)nc),
                                    std::string_view(pk, (size_t)nk), ".AspNetCore.Antiforgery", "TasksCreatedByCookie",
                                    json);
    if (v == formcodec::Verdict::kDecline) return py::none();
    if (v == formcodec::Verdict::kBadToken) return py::make_tuple(false, py::bytes(""));
    return py::make_tuple(true, py::bytes(json));
  });

  // POST Tasks/Edit/{id} (formcodec.hpp edit_task) -> None (the page decides), (False, b"", "")
  // (a bad antiforgery token: 400) or (True, PUT body, task id)
  m.def("frontend_edit_form", [view](py::bytes body, py::bytes cookie, py::bytes key, const std::string& path_id)
            -> py::object {
    std::string json, id;
    auto v = formcodec::edit_task(view(body), view(cookie), view(key), ".AspNetCore.Antiforgery", path_id, json, id);
    if (v == formcodec::Verdict::kDecline) return py::none();
    if (v == formcodec::Verdict::kBadToken) return py::make_tuple(false, py::bytes(""), py::str(""));
    return py::make_tuple(true, py::bytes(json), py::str(id));
  });
  // POST Tasks/Index's form (formcodec.hpp index_post) -> None (the page decides), False (a bad
  // token) or True
  m.def("frontend_index_form", [view](py::bytes body, py::bytes cookie, py::bytes key) -> py::object {
    auto v = formcodec::index_post(view(body), view(cookie), view(key), ".AspNetCore.Antiforgery");
    if (v == formcodec::Verdict::kDecline) return py::none();
    return py::bool_(v == formcodec::Verdict::kOk);
  });

  // state-query response -> (task count, TaskModel JSON array, has a continuation token) or None
  // (taskcodec.hpp query_tasks); `by_created`: ordered by TaskCreatedOn as a DateTime.
  m.def("tasks_from_query", [](py::bytes body, bool by_created, bool descending) -> py::object {
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    std::string out;
    size_t count = 0;
    bool more = false;
    if (!taskcodec::query_tasks(std::string_view(p, (size_t)n), out, count, by_created, &more, descending))
      return py::none();
    return py::make_tuple(count, py::bytes(out), more);
  }, py::arg("body"), py::arg("by_created") = false, py::arg("descending") = false);
  // whether `tasks_from_query` reads this page in its one pass (the store's own layout), for tests
  m.def("tasks_query_in_store_layout", [](py::bytes body) {
    std::string_view b = body.cast<std::string_view>();
    std::string buf;
    std::vector<taskcodec::TaskRow> rows;
    bool token = false;
    return taskcodec::valid_utf8(b) && taskcodec::fast_query_tasks(b, buf, rows, token);
  });

  // A JSON array -> its items re-grouped into arrays of at most `n` items (raw slices, no
  // re-encoding), or None when the text is not a valid JSON array (the processor's chunked
  // markoverdue, services/processor/app.py).
  m.def("json_array_chunks", [](py::bytes body, long n) -> py::object {
    char* pb;
    Py_ssize_t nb;
    if (PyBytes_AsStringAndSize(body.ptr(), &pb, &nb) != 0) throw py::error_already_set();
    std::string_view s(pb, (size_t)nb);
    if (n < 1 || !tt::valid(s)) return py::none();
    const char* p = tt::ws_end(s.data(), s.data() + s.size());
    const char* e = s.data() + s.size();
    if (p >= e || *p != '[') return py::none();
    ++p;
    py::list out;
    std::string cur = "[";
    long in_cur = 0;
    while (true) {
      p = tt::ws_end(p, e);
      if (p < e && *p == ']') break;
      const char* vs = p;
      p = tt::skip_value(p, e);
      if (in_cur) cur += ',';
      cur.append(vs, (size_t)(p - vs));
      if (++in_cur == n) {
        cur += ']';
        out.append(py::bytes(cur));
        cur = "[";
        in_cur = 0;
      }
      p = tt::ws_end(p, e);
      if (p < e && *p == ',') ++p;
    }
    if (in_cur) {
      cur += ']';
      out.append(py::bytes(cur));
    }
    return out;
  });

  // TaskModel JSON -> taskName when it binds within the codec's envelope, else None.
  m.def("task_model_name", [](py::bytes body) -> py::object {
    char* p;
    Py_ssize_t n;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    std::string name;
    if (!taskcodec::task_model_name(std::string_view(p, (size_t)n), name)) return py::none();
    return py::str(name);
  });

  // Columnar query program on the host (cpuscan.hpp): columns = [(uint8 array of the narrow
  // codes, width)], live = uint16 words (1 bit per row), code = int32 [L, 4], bitmaps = uint32.
  // Returns the ascending selected row ids (int32 array).  GIL released while scanning.
  m.def("scan_select",
        [](py::list columns, py::array_t<uint16_t, py::array::c_style> live, int64_t nrows,
           py::array_t<int32_t, py::array::c_style> code, py::array_t<uint32_t, py::array::c_style> bitmaps,
           int threads, bool simd) {
          std::vector<cpuscan::Col> cols;
          std::vector<py::array> keep;
          const int64_t padded = (nrows + 63) / 64 * 64;
          for (auto item : columns) {
            auto t = item.cast<py::tuple>();
            py::array a = t[0].cast<py::array>();
            int w = t[1].cast<int>();
            if (w != 0 && w != 1 && w != 2 && w != 4) throw py::value_error("column width must be 0 (2 bits), 1, 2 or 4");
            if (!(a.flags() & py::array::c_style)) throw py::value_error("columns must be contiguous");
            if ((int64_t)a.nbytes() < (w == 0 ? padded / 4 : padded * w))
              throw py::value_error("column shorter than the padded row count");
            cols.push_back({static_cast<const uint8_t*>(a.data()), w});
            keep.push_back(a);
          }
          if ((int64_t)live.size() * 16 < padded) throw py::value_error("liveness shorter than the padded row count");
          if (code.ndim() != 2 || code.shape(1) != 4) throw py::value_error("code must be [L, 4]");
          cpuscan::Program pg;
          pg.code.assign(code.data(), code.data() + code.size());
          pg.bitmaps.assign(bitmaps.data(), bitmaps.data() + bitmaps.size());
          cpuscan::Selection sel(cols, live.data(), nrows, pg, std::max(1, threads), simd);
          int64_t total;
          {
            py::gil_scoped_release rel;
            total = sel.count();
          }
          // the result is written in place on 2 MiB pages (no copy, few first-touch faults)
          int32_t* dst = static_cast<int32_t*>(cpuscan::huge_alloc((size_t)std::max<int64_t>(total, 1) * sizeof(int32_t)));
          py::capsule owner(dst, [](void* p) { std::free(p); });
          {
            py::gil_scoped_release rel;
            sel.write(dst);
          }
          return py::array_t<int32_t>({(py::ssize_t)total}, {(py::ssize_t)sizeof(int32_t)}, dst, owner);
        },
        py::arg("columns"), py::arg("live"), py::arg("nrows"), py::arg("code"), py::arg("bitmaps"), py::arg("threads"),
        py::arg("simd") = true);

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

  // ops/columnar.py Column: sort ranks of a string dictionary, kept incrementally (strrank.hpp)
  py::class_<StrRanker>(m, "StrRanker")
      .def(py::init<>())
      .def_property_readonly("size", &StrRanker::size)
      .def(
          "extend",
          [](StrRanker& r, py::list values, py::array_t<int64_t, py::array::c_style> ranks) -> int64_t {
            const size_t n0 = r.size(), n = (size_t)PyList_GET_SIZE(values.ptr());
            if (n < n0) return -1;  // the dictionary shrank: the caller starts a new ranker
            if ((size_t)ranks.size() < n || !ranks.writeable()) throw std::invalid_argument("rank buffer too small");
            // every new value first (a non-str, or one UTF-8 cannot carry, leaves nothing changed)
            std::vector<std::string_view> vs;
            vs.reserve(n - n0);
            for (size_t i = n0; i < n; ++i) {
              PyObject* o = PyList_GET_ITEM(values.ptr(), (Py_ssize_t)i);
              if (!PyUnicode_Check(o)) return -1;
              Py_ssize_t len = 0;
              const char* p = PyUnicode_AsUTF8AndSize(o, &len);  // cached in the str: alive with the list
              if (!p) {
                PyErr_Clear();
                return -1;
              }
              vs.emplace_back(p, (size_t)len);
            }
            int64_t* out = ranks.mutable_data();
            return (int64_t)r.extend(vs.size(), [&](size_t i) { return vs[i]; }, out);
          },
          py::arg("values"), py::arg("ranks"));

  py::class_<DocStore>(m, "DocStore")
      .def(py::init<const std::string&, int, size_t>(), py::arg("path") = "", py::arg("fsync_mode") = 0,
           py::arg("index_threshold") = 256)
      // writes from Python return once durable under group commit (fsync_mode 2), as the
      // native front's answers do (a no-op in the other modes)
      .def("set",
           [](DocStore& s, const std::string& key, const std::string& value, const std::optional<std::string>& etag,
              bool first_write, int64_t ttl_ms) {
             std::string e = s.set(key, value, etag, first_write, ttl_ms);
             s.wait_durable();
             return e;
           },
           py::arg("key"), py::arg("value"), py::arg("etag") = std::nullopt, py::arg("first_write") = false,
           py::arg("ttl_ms") = 0, py::call_guard<py::gil_scoped_release>())
      .def("get", &DocStore::get, py::arg("key"))
      .def("delete",
           [](DocStore& s, const std::string& key, const std::optional<std::string>& etag) {
             bool ok = s.del(key, etag);
             s.wait_durable();
             return ok;
           },
           py::arg("key"), py::arg("etag") = std::nullopt, py::call_guard<py::gil_scoped_release>())
      .def("transact",
           [](DocStore& s, const std::vector<TxOp>& ops) {
             s.transact(ops);
             s.wait_durable();
           },
           py::arg("ops"), py::call_guard<py::gil_scoped_release>())
      .def("group_commit", &DocStore::group_commit)
      .def("wait_durable", &DocStore::wait_durable, py::call_guard<py::gil_scoped_release>())
      .def("commit_stats",
           [](DocStore& s) {
             auto c = s.commit_stats();
             py::dict d;
             d["syncs"] = c.syncs;
             d["acks"] = c.acks;
             d["written_bytes"] = c.written;
             d["synced_bytes"] = c.synced;
             d["sync_ms_total"] = c.sync_ms_total;
             d["sync_ms_max"] = c.sync_ms_max;
             return d;
           })
      .def("query", &DocStore::query, py::arg("query"), py::arg("prefix") = "", py::arg("sort_keys") = false,
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
             for (size_t c = 0; c < d.paths.size(); ++c) {
               // every new value a JSON string (timestamps, names): the reader decodes them in
               // one json.loads without checking each text first
               const auto& nv = d.new_values[c];
               const bool all_str =
                   std::all_of(nv.begin(), nv.end(), [](const std::string& v) { return !v.empty() && v[0] == '"'; });
               cols.append(py::make_tuple(d.paths[c], d.dict_from[c], py::cast(nv), arr(d.ids[c]), all_str));
             }
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
              const std::string& prefix, const std::string& token, uint64_t gen,
              std::optional<std::vector<std::string>> sort_paths) -> py::object {
             size_t skipped = 0;
             std::string out;
             const int32_t* p = rows.data();
             size_t n = (size_t)rows.size();
             bool ok;
             {
               py::gil_scoped_release r;
               ok = s.mirror_results(p, n, prefix, token, gen, out, &skipped, sort_paths ? &*sort_paths : nullptr);
             }
             if (!ok) return py::none();  // the rows come from another mirror generation
             return py::make_tuple(py::bytes(out), skipped);
           },
           py::arg("rows"), py::arg("prefix") = "", py::arg("token") = "", py::arg("gen") = 0,
           py::arg("sort_paths") = py::none())
      .def("mirror_stats", &DocStore::mirror_stats)
      .def("set_throughput", &DocStore::set_throughput, py::arg("ru_per_s"), py::arg("ticket_ttl_s") = DocStore::kTicketTtlS)
      .def("charge", [](DocStore& s, double ru, uint64_t ticket, std::string bind, int kind) {
             uint64_t out = 0;
             int64_t wait = s.charge(ru, ticket, out, bind.empty() ? 0 : DocStore::bind_of(bind), kind);
             return py::make_tuple(wait, out);
           }, py::arg("ru"), py::arg("ticket") = 0, py::arg("bind") = "", py::arg("kind") = (int)DocStore::kWrite,
           "(wait_ms, ticket): 0 = admitted; else a 429 whose ticket claims the reserved slot.  `bind`: the "
           "request's identity (method + target [+ query / bulk body]): a retry of the same request without "
           "the ticket claims its due reservation; `kind`: 0 read, 1 write, 2 query, 3 delete")
      .def("debit", &DocStore::debit, py::arg("ru"))
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
             uint64_t seq = b.publish(topic, s, ctype, props, id, ttl_ms, delay_ms);
             b.wait_durable();
             return seq;
           },
           py::arg("topic"), py::arg("body"), py::arg("content_type") = "application/json", py::arg("props") = "{}",
           py::arg("id") = "", py::arg("ttl_ms") = 0, py::arg("delay_ms") = 0)
      .def("send",
           [](Broker& b, const std::string& q, py::bytes body, const std::string& ctype, const std::string& props,
              const std::string& id, int64_t ttl_ms, int64_t delay_ms) {
             std::string s = body;
             py::gil_scoped_release r;
             uint64_t seq = b.send(q, s, ctype, props, id, ttl_ms, delay_ms);
             b.wait_durable();
             return seq;
           },
           py::arg("queue"), py::arg("body"), py::arg("content_type") = "application/json", py::arg("props") = "{}",
           py::arg("id") = "", py::arg("ttl_ms") = 0, py::arg("delay_ms") = 0)
      .def("receive", &Broker::receive, py::arg("path"), py::arg("max_messages") = 1, py::arg("lock_ms") = 0)
      .def("complete",
           [](Broker& b, const std::string& path, const std::string& token) {
             bool ok = b.complete(path, token);
             b.wait_durable();
             return ok;
           },
           py::call_guard<py::gil_scoped_release>())
      .def("abandon",
           [](Broker& b, const std::string& path, const std::string& token, int64_t delay_ms) {
             bool ok = b.abandon(path, token, delay_ms);
             b.wait_durable();
             return ok;
           },
           py::arg("path"), py::arg("token"), py::arg("delay_ms") = 0, py::call_guard<py::gil_scoped_release>())
      .def("dead_letter",
           [](Broker& b, const std::string& path, const std::string& token, const std::string& reason) {
             bool ok = b.dead_letter(path, token, reason);
             b.wait_durable();
             return ok;
           },
           py::arg("path"), py::arg("token"), py::arg("reason") = "", py::call_guard<py::gil_scoped_release>())
      .def("group_commit", &Broker::group_commit)
      .def("commit_stats",
           [](Broker& b) {
             auto c = b.commit_stats();
             py::dict d;
             d["syncs"] = c.syncs;
             d["acks"] = c.acks;
             d["written_bytes"] = c.written;
             d["synced_bytes"] = c.synced;
             d["sync_ms_total"] = c.sync_ms_total;
             d["sync_ms_max"] = c.sync_ms_max;
             return d;
           })
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
      .def(py::init<const std::string&, int, const std::string&, int, const std::string&>(), py::arg("host"),
           py::arg("port"), py::arg("fallback_uds"), py::arg("threads") = 1, py::arg("uds") = "")
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
      .def("set_query_fn",
           [](BackingFront& f, py::function fn) {
             // the worker thread calls back into Python with the GIL; `fn` returns
             // (status, body bytes, [(header, value)]) -- 0 / None: not taken
             // released with the GIL held (stop() may drop it on a thread without it)
             std::shared_ptr<py::function> held(new py::function(std::move(fn)), [](py::function* p) {
               py::gil_scoped_acquire g;
               delete p;
             });
             f.set_query_fn([held](const BackingFront::QueryJob& j) {
               BackingFront::QueryResult out;
               py::gil_scoped_acquire g;
               py::object r = (*held)(j.account, j.db, j.coll, py::bytes(j.body), j.prefix, j.sort_keys, j.traceparent,
                                      j.sent_mono, j.front_mono);
               if (r.is_none()) return out;
               auto t = r.cast<py::tuple>();
               out.status = t[0].cast<int>();
               out.body = t[1].cast<std::string>();
               for (auto h : t[2]) {
                 auto kv = h.cast<py::tuple>();
                 out.headers.emplace_back(kv[0].cast<std::string>(), kv[1].cast<std::string>());
               }
               return out;
             });
           }, py::arg("fn"))
      .def("notify", &BackingFront::notify)
      .def("set_blob_root", &BackingFront::set_blob_root)
      .def("blob_note", &BackingFront::blob_note, py::arg("account"), py::arg("container"), py::arg("name"),
           py::arg("added"), py::call_guard<py::gil_scoped_release>())
      .def("blob_count", &BackingFront::blob_count, py::arg("account"), py::arg("container"), py::arg("prefix") = "",
           py::call_guard<py::gil_scoped_release>())
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
      // a route the I/O thread serves itself (apphost.hpp NativeRoute): kind, settings, the
      // latency histogram's buckets -> route id
      .def("add_route", &apphost::AppHost::add_route, py::arg("server"), py::arg("kind"), py::arg("cfg"),
           py::arg("bounds"), py::call_guard<py::gil_scoped_release>())
      // [(route id, status, count, latency sum s, bucket counts)] since the last call
      .def("route_stats", [](apphost::AppHost& h) {
        auto st = h.take_route_stats();
        py::list out;
        for (auto& x : st) out.append(py::make_tuple(x.route, x.status, x.n, x.sum, x.buckets));
        return out;
      })
      // ops: [(0, token, status, headers, body) | (1, id, endpoint, method, target, headers, body, timeout) |
      //       (2, id, endpoint, "", grpc_path, metadata, message, timeout)]
      .def("submit",
           [](apphost::AppHost& h, py::list ops) {
             std::vector<apphost::AppHost::Op> v;
             Py_ssize_t n = PyList_GET_SIZE(ops.ptr());
             v.reserve((size_t)n);
             for (Py_ssize_t i = 0; i < n; ++i) {
               py::object t = seq_fast(PyList_GET_ITEM(ops.ptr(), i), "an operation must be a tuple");
               Py_ssize_t len = PySequence_Fast_GET_SIZE(t.ptr());
               PyObject** f = PySequence_Fast_ITEMS(t.ptr());
               if (len < 2) throw py::value_error("operation too short");
               apphost::AppHost::Op op;
               long long kind = need_int(f[0], "operation kind");
               op.is_request = kind == 1 || kind == 2;
               op.is_grpc = kind == 2;
               op.id = (uint64_t)need_int(f[1], "operation id");
               if (!op.is_request) {
                 if (len != 5) throw py::value_error("respond operation: (0, token, status, headers, body)");
                 op.status = (int)need_int(f[2], "status");
                 op.headers = header_list_fast(f[3]);
                 op.body = body_of(f[4]);
               } else {
                 if (len != 8) throw py::value_error("request operation: (1, id, endpoint, method, target, headers, body, timeout)");
                 op.endpoint = std::string(need_str(f[2], "endpoint"));
                 op.method = std::string(need_str(f[3], "method"));
                 op.target = std::string(need_str(f[4], "target"));
                 op.headers = header_list_fast(f[5]);
                 op.body = body_of(f[6]);
                 op.timeout_s = PyFloat_AsDouble(f[7]);
                 if (op.timeout_s == -1.0 && PyErr_Occurred()) throw py::error_already_set();
               }
               v.push_back(std::move(op));
             }
             h.submit(std::move(v));
           })
      // [(0, token, server, method, target, http10, headers, body) | (1, id, status, headers, body) |
      //  (2, id, errno, message)] (+ each event's queue time, monotonic seconds, with drain_times)
      .def("drain_times", [](apphost::AppHost& h) {
        auto evs = h.drain();
        return events_to_py(evs, true);
      })
      .def("drain", [](apphost::AppHost& h) {
        auto evs = h.drain();
        return events_to_py(evs, false);
      });
}
