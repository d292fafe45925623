// Sort ranks of a growing dictionary of strings -- the column mirror's timestamps, names and
// e-mails (ops/columnar.py Column._string_ranks, the GPU sort plan's rank tables).
//
// A dictionary id's rank is its position in the sorted dictionary (distinct values, ranks from
// 1).  Values only ever get appended; new timestamps arrive nearly in order, so each update
// sorts the new values alone and merges them into the tail of the order they land in: O(tail
// + new log new), not a sort of the dictionary.  The strings are kept as UTF-8 in one arena
// (no allocation per value); UTF-8 byte order is code point order, which is Python's str order.
//
// The ranks are written into a caller-owned int64 buffer (a numpy array the caller grows), so
// the caller's views of it stay valid: only the ranks of ids whose position moved are written.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <string>
#include <string_view>
#include <vector>

namespace tt {

class StrRanker {
 public:
  size_t size() const { return off_.size(); }

  // Append `utf8` values (ids size() .. size() + count - 1) and update `ranks` (capacity >=
  // the new size).  Returns the first id whose rank may have changed (the old size when every
  // new value sorts after the old ones).
  template <class Get>
  size_t extend(size_t count, Get&& get, int64_t* ranks) {
    const size_t n0 = off_.size(), n = n0 + count;
    for (size_t i = 0; i < count; ++i) {
      std::string_view v = get(i);
      off_.push_back(arena_.size());
      len_.push_back((uint32_t)v.size());
      arena_.append(v);
    }
    if (count == 0) return n0;
    std::vector<uint32_t> nw(count);
    std::iota(nw.begin(), nw.end(), (uint32_t)n0);
    auto less = [this](uint32_t a, uint32_t b) { return view(a) < view(b); };
    if (!std::is_sorted(nw.begin(), nw.end(), less)) std::stable_sort(nw.begin(), nw.end(), less);
    // where the smallest new value lands: only the old values from there on move
    size_t pos0 = n0;
    if (n0 && !less(sorted_.back(), nw[0]))
      pos0 = (size_t)(std::lower_bound(sorted_.begin(), sorted_.end(), nw[0], less) - sorted_.begin());
    size_t lo = n0;
    if (pos0 == n0) {
      sorted_.insert(sorted_.end(), nw.begin(), nw.end());
    } else {
      std::vector<uint32_t> tail(sorted_.begin() + (long)pos0, sorted_.end());
      for (uint32_t id : tail) lo = std::min<size_t>(lo, id);
      sorted_.resize(pos0);
      // an old value equal to a new one stays first (the order a stable sort of old-then-new gives)
      std::merge(tail.begin(), tail.end(), nw.begin(), nw.end(), std::back_inserter(sorted_), less);
    }
    for (size_t p = pos0; p < n; ++p) ranks[sorted_[p]] = (int64_t)p + 1;
    return lo;
  }

 private:
  std::string arena_;
  std::vector<uint64_t> off_;
  std::vector<uint32_t> len_;
  std::vector<uint32_t> sorted_;  // ids in value order

  std::string_view view(uint32_t id) const { return std::string_view(arena_.data() + off_[id], len_[id]); }
};

}  // namespace tt
