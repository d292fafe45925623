// The store's bulk update (the overdue sweep's markoverdue save) in isolation: 400k task
// documents, then 300 bulk saves of 128 documents, and 128 single gets, timed.
//   mode 0: no column mirror; 1: mirror on, isOverDue flips (the sweep's update);
//   2: mirror on, only taskName changes (every mirrored id carried over).
// The set_many time covers the lock hold plus freeing the replaced versions after it.
//   g++ -O3 -std=c++17 -I aca_dotnet_workshop_amd/native/src scripts/store_bulk_bench.cpp \
//       -o /tmp/store_bulk_bench -lpthread -lssl -lcrypto && /tmp/store_bulk_bench 1
#include "docstore.hpp"
#include <chrono>
#include <cstdio>
using namespace tt;
static std::string doc(int i, bool overdue, const char* name = "Task") {
  char b[512];
  snprintf(b, sizeof b, "{\"taskId\":\"%08x-0000-4000-8000-%012d\",\"taskName\":\"%s %d\",\"taskCreatedBy\":\"bench@bench.local\",\"taskCreatedOn\":\"2026-10-18T12:%02d:%02d.%06d\",\"taskDueDate\":\"2026-%02d-%02dT00:00:00\",\"taskAssignedTo\":\"a%d@x.com\",\"isCompleted\":false,\"isOverDue\":%s}",
           i, i, name, i, (i / 60) % 60, i % 60, i, 1 + i % 12, 1 + i % 28, i % 97, overdue ? "true" : "false");
  return b;
}
static std::string key(int i) { char b[64]; snprintf(b, sizeof b, "tasksmanager-backend-api||%08x-0000-4000-8000-%012d", i, i); return b; }
int main(int argc, char** argv) {
  int mode = atoi(argv[1]);  // 0 no mirror, 1 mirror + isOverDue flip, 2 mirror + name change only
  DocStore s("", 0, 256);
  if (mode) s.mirror_enable({"taskDueDate", "isCompleted", "isOverDue", "taskCreatedOn"});
  const int N = 400000;
  for (int i = 0; i < N; ++i) s.set(key(i), doc(i, false), std::nullopt, false, 0);
  std::vector<std::vector<DocStore::BulkItem>> all;
  int reps = 300;
  for (int r = 0; r < reps; ++r) {
    std::vector<DocStore::BulkItem> items;
    for (int j = 0; j < 128; ++j) {
      int i = (r * 7919 + j * 3001) % N;
      DocStore::BulkItem it; it.key = key(i); it.value = mode == 2 ? doc(i, false, "Renamed") : doc(i, true);
      it.parsed = parse(it.value); it.have_parsed = true;
      items.push_back(std::move(it));
    }
    all.push_back(std::move(items));
  }
  std::vector<std::string> gk; for (int j = 0; j < 128; ++j) gk.push_back(key((j * 3001 + 17) % N));
  auto a = std::chrono::steady_clock::now();
  for (auto& items : all) s.set_many(items);
  double d = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
  auto b = std::chrono::steady_clock::now();
  size_t n = 0;
  for (int r = 0; r < reps; ++r) for (auto& k : gk) { auto g = s.get(k); n += g ? g->first.size() : 0; }
  double dg = std::chrono::duration<double>(std::chrono::steady_clock::now() - b).count();
  printf("mode %d: set_many(128) pre-parsed %.1f us (%.2f us/doc); 128 gets %.1f us\n", mode, d / reps * 1e6, d / reps / 128 * 1e6, dg / reps * 1e6);
}
