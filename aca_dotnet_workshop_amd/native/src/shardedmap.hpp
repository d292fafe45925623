// String-keyed hash map split into independently growing shards.
//
// A std::unordered_map grows by relinking every node into a bucket array about twice as large,
// all at once: for the document store's 350k-document collection (or a column dictionary with a
// value per document) that is ~20-50 ms during which the store lock is held and every front
// thread waits on it (profiles/r4_sweep_tail.md).  Here each of kShards maps grows on its own,
// so a growth step relinks 1/kShards of the entries.  Keys spread evenly over the shards, so
// shards with equal load limits would all reach them within the same few thousand inserts: the
// whole collection relinked in one burst after all, only in 1/kShards slices.  Each shard has its
// own load limit instead, 2^(-s/kShards) for shard s (0.5-1.0), so the shards' growth points
// spread evenly over every doubling of the collection.  Node-based like the maps it is made of:
// references and pointers to elements stay valid until the element is erased (the column
// mirror keeps pointers to the keys).  Iteration order is unspecified, as for unordered_map.
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <utility>

namespace tt {

template <class V, size_t kShards = 64>
class ShardedMap {
  static_assert((kShards & (kShards - 1)) == 0, "kShards must be a power of two");
  using Inner = std::unordered_map<std::string, V>;

 public:
  using value_type = typename Inner::value_type;

  ShardedMap() {
    for (size_t s = 0; s < kShards; ++s) shards_[s].max_load_factor((float)std::exp2(-(double)s / (double)kShards));
  }

  class iterator {
   public:
    iterator() = default;
    value_type& operator*() const { return *it_; }
    value_type* operator->() const { return &*it_; }
    iterator& operator++() {
      ++it_;
      skip_empty();
      return *this;
    }
    bool operator==(const iterator& o) const { return shard_ == o.shard_ && (shard_ == kShards || it_ == o.it_); }
    bool operator!=(const iterator& o) const { return !(*this == o); }

   private:
    friend class ShardedMap;
    iterator(ShardedMap* m, size_t shard, typename Inner::iterator it) : m_(m), shard_(shard), it_(it) {}
    void skip_empty() {
      while (shard_ < kShards && it_ == m_->shards_[shard_].end()) {
        if (++shard_ < kShards) it_ = m_->shards_[shard_].begin();
      }
    }
    ShardedMap* m_ = nullptr;
    size_t shard_ = kShards;
    typename Inner::iterator it_{};
  };

  iterator begin() {
    iterator it(this, 0, shards_[0].begin());
    it.skip_empty();
    return it;
  }
  iterator end() { return iterator(this, kShards, {}); }

  iterator find(const std::string& k) {
    size_t s = shard_of(k);
    auto it = shards_[s].find(k);
    return it == shards_[s].end() ? end() : iterator(this, s, it);
  }
  size_t count(const std::string& k) const { return shards_[shard_of(k)].count(k); }
  V& operator[](const std::string& k) { return shards_[shard_of(k)][k]; }
  template <class... A>
  std::pair<iterator, bool> emplace(const std::string& k, A&&... a) {
    size_t s = shard_of(k);
    auto [it, fresh] = shards_[s].try_emplace(k, std::forward<A>(a)...);
    return {iterator(this, s, it), fresh};
  }
  void erase(iterator it) { shards_[it.shard_].erase(it.it_); }
  size_t size() const {
    size_t n = 0;
    for (auto& s : shards_) n += s.size();
    return n;
  }
  bool empty() const { return size() == 0; }
  size_t bucket_count(size_t shard) const { return shards_[shard].bucket_count(); }
  static constexpr size_t shards() { return kShards; }
  void clear() {
    for (auto& s : shards_) s.clear();
  }

 private:
  // the shard from a cheap fold of the key's bytes (FNV-1a over at most its last 24 bytes --
  // generated ids and timestamps differ at the end); the shard's own map hashes the whole key
  static size_t shard_of(const std::string& k) {
    uint64_t h = 1469598103934665603ull;
    size_t from = k.size() > 24 ? k.size() - 24 : 0;
    for (size_t i = from; i < k.size(); ++i) h = (h ^ (unsigned char)k[i]) * 1099511628211ull;
    return (size_t)(h ^ (h >> 29)) & (kShards - 1);
  }

  Inner shards_[kShards];
};

}  // namespace tt
