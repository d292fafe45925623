// Stress program for the app-process native host (src/apphost.hpp), built under ThreadSanitizer
// and ASan+UBSan by tests/test_native_sanitizers.py.
//
// The main thread plays the Python side: it waits on event_fd(), drains events, answers every
// server request (submit(respond)) and issues client requests (submit(request)) to the host's
// own listener over a Unix socket and TCP, so the I/O thread runs server and client paths
// concurrently with the submitting thread.  Every response must carry the body its request
// asked for; a refused endpoint must produce an ERROR event.
//
//   apphost_stress <requests> <inflight> <sock-path>
#include <poll.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>

#include "../src/apphost.hpp"

using tt::apphost::AppHost;
using tt::apphost::Event;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const int total = argc > 1 ? std::atoi(argv[1]) : 20000;
  const int inflight = argc > 2 ? std::atoi(argv[2]) : 64;
  const std::string sock = argc > 3 ? argv[3] : "/tmp/apphost_stress.sock";

  AppHost host;
  host.listen(1, "unix:" + sock);
  int port = host.listen(1, "tcp:127.0.0.1:0");
  host.start();
  const std::string eps[2] = {"unix:" + sock, "tcp:127.0.0.1:" + std::to_string(port)};

  std::map<uint64_t, std::string> expect;  // client id -> expected body
  uint64_t next_id = 1;
  int sent = 0, done = 0, served = 0;
  auto issue = [&](std::vector<AppHost::Op>& ops) {
    AppHost::Op op;
    op.is_request = true;
    op.id = next_id++;
    op.endpoint = eps[op.id % 2];
    op.method = (op.id % 3 == 0) ? "GET" : "POST";
    op.target = "/echo/" + std::to_string(op.id);
    op.headers = {{"x-id", std::to_string(op.id)}};
    op.body = op.method == "POST" ? std::string(op.id % 97 * 13, 'a' + (char)(op.id % 26)) : "";
    op.timeout_s = 30;
    expect[op.id] = op.method + " " + op.target + " " + op.body;
    ops.push_back(std::move(op));
    ++sent;
  };

  std::vector<AppHost::Op> ops;
  for (int i = 0; i < inflight && sent < total; ++i) issue(ops);
  host.submit(std::move(ops));

  while (done < total) {
    pollfd p{host.event_fd(), POLLIN, 0};
    if (::poll(&p, 1, 10000) <= 0) return fail("timed out waiting for events");
    std::vector<AppHost::Op> out;
    for (auto& e : host.drain()) {
      if (e.kind == Event::REQUEST) {
        AppHost::Op r;
        r.id = e.id;
        r.status = 200;
        r.headers = {{"content-type", "text/plain"}};
        r.body = e.msg.method + " " + e.msg.target + " " + e.msg.body;
        auto* xid = e.msg.header("x-id");
        if (!xid || e.msg.target != "/echo/" + *xid) return fail("request header/target mismatch");
        out.push_back(std::move(r));
        ++served;
      } else if (e.kind == Event::RESPONSE) {
        auto it = expect.find(e.id);
        if (it == expect.end()) return fail("response for an unknown id");
        if (e.msg.status != 200 || e.msg.body != it->second) return fail("response body mismatch");
        expect.erase(it);
        ++done;
        if (sent < total) issue(out);
      } else {
        return fail("unexpected client error");
      }
    }
    if (!out.empty()) host.submit(std::move(out));
  }
  if (served != total) return fail("server count mismatch");

  // a refused endpoint surfaces as an ERROR event
  std::vector<AppHost::Op> bad(1);
  bad[0].is_request = true;
  bad[0].id = 999999999;
  bad[0].endpoint = "unix:" + sock + ".missing";
  bad[0].method = "GET";
  bad[0].target = "/";
  host.submit(std::move(bad));
  bool got_error = false;
  for (int i = 0; i < 50 && !got_error; ++i) {
    pollfd p{host.event_fd(), POLLIN, 0};
    ::poll(&p, 1, 100);
    for (auto& e : host.drain())
      if (e.kind == Event::ERROR && e.id == 999999999) got_error = true;
  }
  if (!got_error) return fail("no error event for a missing socket");
  host.close_server(1);
  host.stop();
  std::printf("apphost ok: %d requests, %d inflight\nALL OK\n", total, inflight);
  return 0;
}
