// Stress program for the pipelined client connections (src/evhttp.hpp PipeConn,
// Client::request_pipelined) and the answers batched per read (ServerConn::parse), built under
// ThreadSanitizer and ASan+UBSan by tests/test_native_sanitizers.py.
//
// One loop serves a Unix socket whose handler answers some requests at once, some from a timer
// (out of arrival order, so the in-order slots matter) and now and then drops every connection; the
// same loop's client keeps `inflight` pipelined requests going.  Every answer must carry the id
// its request sent; a dropped connection must fail the requests still on it (with an error,
// never another request's answer) and later requests must get through on new connections; and
// every request must complete exactly once.
//
//   pipe_stress <requests> <inflight> <sock-path>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <unordered_map>

#include "../src/evhttp.hpp"

using namespace tt::ev;

int main(int argc, char** argv) {
  const int total = argc > 1 ? std::atoi(argv[1]) : 20000;
  const int inflight = argc > 2 ? std::atoi(argv[2]) : 64;
  const std::string sock = argc > 3 ? argv[3] : "/tmp/pipe_stress.sock";
  ::unlink(sock.c_str());

  Loop loop;
  std::mt19937 rng(7);
  int closes = 0;
  std::vector<std::weak_ptr<ServerConn>> conns;
  Handler h = [&](Message&& m, Reply r) {
    const std::string id = m.target.substr(m.target.rfind('/') + 1);
    const int n = std::atoi(id.c_str());
    if (n % 97 == 0) {  // a slow answer: the ones queued behind it on this connection wait
      loop.call_later(0.002, [r, id] { r.send(200, {{"x-id", id}}, "late " + id); });
    } else if (n % 1331 == 0) {  // the server drops every connection: what is in flight fails
      ++closes;
      loop.defer([&] {
        for (auto& w : conns)
          if (auto c = w.lock()) loop.remove(c.get());
        conns.clear();
      });
    } else {
      r.send(200, {{"x-id", id}}, "now " + id + " " + m.body);
    }
  };
  Endpoint ep = Endpoint::parse("unix:" + sock);
  std::shared_ptr<IoObj> lst;
  listen_on(loop, ep, h, false, &lst);
  std::static_pointer_cast<Listener>(lst)->on_accept = [&](const std::shared_ptr<ServerConn>& c) { conns.push_back(c); };
  Client client(loop);

  std::unordered_map<int, std::string> pending;  // id -> body sent
  int next = 1, ok = 0, failed = 0, bad = 0;
  std::function<void()> issue = [&] {
    if (next > total) return;
    const int id = next++;
    std::string body(rng() % 300, (char)('a' + id % 26));
    pending[id] = body;
    client.request_pipelined(ep, "POST", "/echo/" + std::to_string(id), {{"content-type", "text/plain"}}, body, 30,
                             [&, id](ClientResult&& res) {
                               auto it = pending.find(id);
                               if (it == pending.end()) {
                                 ++bad;  // completed twice
                               } else {
                                 if (res.err) {
                                   ++failed;
                                 } else {
                                   const std::string* x = res.resp.header("x-id");
                                   const std::string sid = std::to_string(id);
                                   const bool match =
                                       x && *x == sid &&
                                       (res.resp.body == "now " + sid + " " + it->second ||
                                        res.resp.body == "late " + sid);
                                   if (match) ++ok;
                                   else ++bad;
                                 }
                                 pending.erase(it);
                               }
                               if (ok + failed + bad >= total) loop.stop();
                               else issue();
                             });
  };
  for (int i = 0; i < inflight; ++i) issue();
  loop.call_later(120.0, [&] {
    std::fprintf(stderr, "timeout: ok %d failed %d bad %d pending %zu\n", ok, failed, bad, pending.size());
    loop.stop();
  });
  loop.run();
  ::unlink(sock.c_str());
  std::printf("ok %d failed %d bad %d pending %zu closes %d pipelined %llu\n", ok, failed, bad, pending.size(), closes,
              (unsigned long long)client.pipelined());
  // every request completed exactly once, every answer was its own, and only requests caught on
  // a connection the server closed failed
  if (bad || !pending.empty() || ok + failed != total || failed > closes * inflight || (closes && !failed) ||
      ok < total - closes * inflight || client.pipelined() == 0) {
    std::printf("FAIL\n");
    return 1;
  }
  std::printf("ALL OK\n");
  return 0;
}
