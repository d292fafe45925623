// Concurrency stress test for the native engines, built with -fsanitize=thread or
// -fsanitize=address,undefined by tests/test_native_sanitizers.py (host code only).
//
// Several threads hammer one DocStore (set / get / delete / transactions with ETags /
// indexed and scanning queries) and one Broker (publish / receive / complete / abandon /
// renew / dead-letter / counts) at the same time, the way the backing-services process uses
// them with the GIL released.  Invariants checked at the end:
//   * every published message is either completed or dead-lettered exactly once;
//   * the store's document count equals the number of keys the writers left alive.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../src/backingfront.hpp"
#include "../src/broker.hpp"
#include "../src/docstore.hpp"
#include "../src/httpparse.hpp"

using namespace tt;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  std::string log_path = argc > 3 ? argv[3] : "";

  // ---------------------------------------------------------------- document store
  {
    DocStore store(log_path, 0, 64);
    std::atomic<int> conflicts{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
      ts.emplace_back([&, t] {
        std::mt19937 rng(1234 + t);
        for (int i = 0; i < iters; ++i) {
          std::string key = "k" + std::to_string(rng() % 200);
          std::string doc = "{\"owner\":\"u" + std::to_string(rng() % 10) + "\",\"n\":" + std::to_string(i) +
                            ",\"done\":" + (rng() % 2 ? "true" : "false") + "}";
          switch (rng() % 6) {
            case 0: {
              auto cur = store.get(key);
              try {
                store.set(key, doc, cur ? std::optional<std::string>(cur->second) : std::nullopt, !cur, 0);
              } catch (const EtagMismatch&) {
                conflicts++;
              }
              break;
            }
            case 1:
              store.set(key, doc, std::nullopt, false, 0);
              break;
            case 2:
              try {
                store.del(key, std::nullopt);
              } catch (const EtagMismatch&) {
              }
              break;
            case 3:
              store.query("{\"filter\":{\"EQ\":{\"owner\":\"u3\"}},\"sort\":[{\"key\":\"n\",\"order\":\"DESC\"}]}", "");
              break;
            case 4:
              store.query("{\"filter\":{\"OR\":[{\"GT\":{\"n\":100}},{\"EQ\":{\"done\":true}}]},\"page\":{\"limit\":5}}", "");
              break;
            default: {
              std::vector<TxOp> ops(2);
              ops[0].key = key;
              ops[0].value = doc;
              ops[1].key = "k" + std::to_string(rng() % 200);
              ops[1].is_delete = true;
              try {
                store.transact(ops);
              } catch (const EtagMismatch&) {
              }
            }
          }
        }
      });
    }
    for (auto& th : ts) th.join();
    auto keys = store.keys("", 0);
    if (keys.size() != store.size()) return fail("docstore key count");
    for (auto& k : keys)
      if (!store.get(k)) return fail("docstore key without document");
    std::printf("docstore ok: %zu docs, %d etag conflicts\n", store.size(), conflicts.load());
  }

  // ---------------------------------------------------------------- broker
  {
    Broker broker;
    QueueOptions o;
    o.lock_ms = 5;
    o.max_delivery = 4;
    broker.create_subscription("topic", "sub", o);
    const std::string path = "topic/subscriptions/sub";
    const int producers = threads / 2 > 0 ? threads / 2 : 1;
    const int per_producer = iters;
    std::atomic<long> completed{0};
    std::atomic<bool> done_producing{false};
    std::vector<std::thread> ts;
    for (int p = 0; p < producers; ++p)
      ts.emplace_back([&, p] {
        for (int i = 0; i < per_producer; ++i)
          broker.publish("topic", "m" + std::to_string(p) + "-" + std::to_string(i), "text/plain", "{}", "", 0, 0);
      });
    for (int c = 0; c < threads - producers + 1; ++c)
      ts.emplace_back([&, c] {
        std::mt19937 rng(99 + c);
        int idle = 0;
        while (idle < 200) {
          auto msgs = broker.receive(path, 8, 0);
          if (msgs.empty()) {
            if (done_producing) ++idle;
            std::this_thread::yield();
            continue;
          }
          idle = 0;
          for (auto& m : msgs) {
            switch (rng() % 8) {
              case 0: broker.abandon(path, m.lock_token, 0); break;
              case 1: broker.renew(path, m.lock_token, 0); broker.complete(path, m.lock_token) && ++completed; break;
              case 2: break;  // let the lock expire -> redelivery
              default:
                if (broker.complete(path, m.lock_token)) ++completed;
            }
          }
          broker.counts(path);
        }
      });
    for (int p = 0; p < producers; ++p) ts[p].join();
    done_producing = true;
    for (size_t i = producers; i < ts.size(); ++i) ts[i].join();
    // drain what is left (locks of abandoned/expired messages may still be pending)
    for (int spin = 0; spin < 2000; ++spin) {
      auto msgs = broker.receive(path, 64, 0);
      for (auto& m : msgs)
        if (broker.complete(path, m.lock_token)) ++completed;
      auto [a, s, l, d, e, c, r] = broker.counts(path);
      if (a == 0 && s == 0 && l == 0) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    auto [a, s, l, d, e, c, r] = broker.counts(path);
    long total = (long)producers * per_producer;
    if ((long)c != completed.load()) return fail("broker completed counter mismatch");
    if ((long)c + (long)d != total) {
      std::fprintf(stderr, "completed=%ld dead=%zu total=%ld active=%zu locked=%zu\n", (long)c, d, total, a, l);
      return fail("broker lost or duplicated messages");
    }
    std::printf("broker ok: %ld completed, %zu dead-lettered of %ld\n", (long)c, d, total);
  }

  // ---------------------------------------------------------------- backing front
  // HTTP clients on several threads against the native front's loop thread while the
  // "Python" thread reconfigures it (policy, notify) and builds / reads the column mirror.
  {
    DocStore store;
    Broker broker, storage;
    QueueOptions o;
    broker.create_subscription("t", "s", o);
    BackingFront front("127.0.0.1", 0, "/nonexistent/fallback.sock", 3);
    front.attach_store("a", "d", "c", &store);
    front.attach_broker("ns", &broker);
    front.attach_broker("storage-sa", &storage);  // the storage queue and blob routes too
    std::string blob_root = std::string(argc > 3 ? argv[3] : "/tmp/stress") + ".blobs";
    front.set_blob_root(blob_root);
    int port = front.port();
    auto http = [port](const std::string& req) {
      int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)port);
      inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
      std::string out;
      if (::connect(fd, (sockaddr*)&a, sizeof a) == 0) {
        ::send(fd, req.data(), req.size(), MSG_NOSIGNAL);
        char buf[8192];
        ssize_t n;
        while ((n = ::recv(fd, buf, sizeof buf, 0)) > 0) out.append(buf, (size_t)n);
      }
      ::close(fd);
      return out;
    };
    std::atomic<int> ok{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t)
      ts.emplace_back([&, t] {
        for (int i = 0; i < 100; ++i) {
          std::string k = "k" + std::to_string((t * 100 + i) % 37), body = "{\"v\":" + std::to_string(i) + "}";
          std::string r1 = http("PUT /cosmos/a/d/c/docs/" + k + " HTTP/1.1\r\nContent-Length: " +
                                std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body);
          std::string r2 = http("GET /cosmos/a/d/c/docs/" + k + " HTTP/1.1\r\nConnection: close\r\n\r\n");
          std::string r3 = http("POST /servicebus/ns/topics/t/messages HTTP/1.1\r\nContent-Length: 2\r\n"
                                "Connection: close\r\n\r\n{}");
          std::string r4 = http("POST /servicebus/ns/receive?entity=t/subscriptions/s&max=4&waitMs=1 HTTP/1.1\r\n"
                                "Connection: close\r\n\r\n");
          std::string r5 = http("POST /storage/sa/queues/q/messages HTTP/1.1\r\nContent-Length: 2\r\n"
                                "Connection: close\r\n\r\nhi");
          std::string r6 = http("GET /storage/sa/queues/q/messages?numofmessages=2&visibilityMs=1&waitMs=1 HTTP/1.1\r\n"
                                "Connection: close\r\n\r\n");
          std::string r7 = http("PUT /storage/sa/blobs/box/d" + std::to_string(t) + "/b" + std::to_string(i % 9) +
                                ".json HTTP/1.1\r\nContent-Length: 2\r\nConnection: close\r\n\r\n{}");
          std::string r8 = http("GET /storage/sa/blobs/box?count=true HTTP/1.1\r\nConnection: close\r\n\r\n");
          if (r1.rfind("HTTP/1.1 ", 0) == 0 && r3.rfind("HTTP/1.1 201", 0) == 0 && r4.rfind("HTTP/1.1 200", 0) == 0 &&
              r5.rfind("HTTP/1.1 201", 0) == 0 && r6.rfind("HTTP/1.1 200", 0) == 0 && r7.rfind("HTTP/1.1 201", 0) == 0 &&
              r8.rfind("HTTP/1.1 200", 0) == 0)
            ok++;
        }
      });
    for (int i = 0; i < 200; ++i) {
      front.set_policy(i % 2 ? "open" : "open", {{"cosmos/a", "key"}}, {{"p", "cosmos/a", {"cosmos.read"}}});
      front.notify("ns", "t/subscriptions/s");
      front.blob_note("sa", "box", "py" + std::to_string(i % 5) + ".json", i % 3 != 0);  // Python's puts / deletes
      (void)front.blob_count("sa", "box", i % 2 ? "d1/" : "");
      // the columnar mirror is built and read while the front's threads keep writing natively
      if (i == 50) store.mirror_enable({"v"});
      if (i > 50) {
        MirrorDelta d = store.mirror_delta(i % 7 ? 0 : 2, 0, 0, {});
        int32_t rows[2] = {0, (int32_t)(d.n ? d.n - 1 : 0)};
        std::string res;
        store.mirror_results(rows, 2, "", "", d.gen, res);
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    for (auto& th : ts) th.join();
    front.stop();
    std::error_code ec;
    std::filesystem::remove_all(blob_root, ec);
    if (ok.load() < 100) return fail("backing front served too few requests");
    std::printf("backing front ok: %d request rounds\n", ok.load());
  }

  // ---------------------------------------------------------------- http head parser
  {
    auto h = parse_head("GET /x HTTP/1.1\r\nHost: a\r\nX-Y:  z \r\n");
    if (h.a != "GET" || h.headers.size() != 2 || h.headers[1].second != "z") return fail("http parse");
    try {
      parse_head("garbage");
      return fail("http parse accepted garbage");
    } catch (const std::invalid_argument&) {
    }
  }
  std::printf("ALL OK\n");
  return 0;
}
