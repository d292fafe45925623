// Micro-benchmark of the overdue sweep's bulk save inside the document store: a collection of
// N task documents (column mirror on, creator index built, append log on), then R rounds of
// `set_many` over B of them (the ~700 tasks one sweep marks overdue), timed per phase.
//
//   g++ -O2 -std=c++17 -pthread bulk_bench.cpp -o /tmp/bulk_bench && /tmp/bulk_bench 400000 700 20 /tmp/bb.log
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../src/backingfront.hpp"
#include "../src/docstore.hpp"

using namespace tt;
using clk = std::chrono::steady_clock;

static std::string task_json(int i, bool overdue) {
  char buf[512];
  std::snprintf(buf, sizeof buf,
                "{\"taskId\":\"%08x-1c2d-4e5f-8a9b-%012d\",\"taskName\":\"task %d\",\"taskCreatedBy\":\"user%d@mail.com\","
                "\"taskCreatedOn\":\"2026-10-17T04:%02d:%02d.%07d\",\"taskDueDate\":\"2026-10-%02dT00:00:00\","
                "\"taskAssignedTo\":\"assignee%d@mail.com\",\"isCompleted\":false,\"isOverDue\":%s}",
                i, i, i, i % 97, (i / 60) % 60, i % 60, i % 9999999, 1 + i % 28, i % 13, overdue ? "true" : "false");
  return buf;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 400000;
  const int b = argc > 2 ? std::atoi(argv[2]) : 700;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 20;
  const std::string log = argc > 4 ? argv[4] : "";
  DocStore store(log, 0, 256);
  for (int i = 0; i < n; ++i) store.set("tasks||" + std::to_string(i), task_json(i, false), std::nullopt, false, 0);
  store.mirror_enable({std::string("\x00keyprefix", 10), "taskDueDate", "isCompleted", "isOverDue", "taskCreatedOn"});
  store.query("{\"filter\":{\"EQ\":{\"taskCreatedBy\":\"user1@mail.com\"}}}", "tasks||");  // builds the index
  double parse_us = 0, set_us = 0;
  for (int r = 0; r < rounds; ++r) {
    std::string body = "[";
    for (int j = 0; j < b; ++j) {
      int i = (r * b + j) * 7 % n;
      if (j) body += ",";
      body += "{\"key\":\"tasks||" + std::to_string(i) + "\",\"value\":" + task_json(i, true) + "}";
    }
    body += "]";
    auto t0 = clk::now();
    std::vector<DocStore::BulkItem> batch;  // the backing front's scan of the data plane's body
    if (!scan_bulk_items(body, batch)) { std::fprintf(stderr, "scan failed\n"); return 1; }
    auto t1 = clk::now();
    auto res = store.set_many(batch);
    auto t2 = clk::now();
    if (res.size() != (size_t)b || res[0].err) { std::fprintf(stderr, "bulk failed\n"); return 1; }
    parse_us += std::chrono::duration<double, std::micro>(t1 - t0).count();
    set_us += std::chrono::duration<double, std::micro>(t2 - t1).count();
  }
  std::printf("{\"docs\": %d, \"batch\": %d, \"rounds\": %d, \"body_parse_us_per_doc\": %.2f, \"set_many_us_per_doc\": %.2f}\n",
              n, b, rounds, parse_us / rounds / b, set_us / rounds / b);
  return 0;
}
