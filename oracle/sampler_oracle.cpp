// oracle/sampler_oracle.cpp -- TEST INFRASTRUCTURE ONLY.
//
// initSampler's non-IID bucket construction (Server/src/main/c++/
// cppNN_backend.cpp:387, :411-470) restated as the reference compiles it: C++11,
// the labels' index order from sort_indexes (:116-127, std::sort over size_t
// indices), and std::random_shuffle -- the library's own, not a restatement --
// with the reference's generator [](int i) { return std::rand() % i; } over
// libc rand() after srand(seed). The product (fleet_amd/csrc/sampler_state.cpp)
// restates random_shuffle's loop; this checker runs the real one.
//
// Parity: pinned to the reference's own call sequence on the image's libstdc++
// and glibc (the reference's results on its authors' toolchain depend on theirs:
// std::sort's order of equal labels and rand()'s sequence are implementation
// choices). Only tests/ use this library.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <numeric>
#include <vector>

namespace {

template <typename T>
std::vector<size_t> sort_indexes(const std::vector<T>& v) {  // :116-127
  std::vector<size_t> idx(v.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::sort(idx.begin(), idx.end(), [&v](size_t i1, size_t i2) { return v[i1] < v[i2]; });
  return idx;
}

}  // namespace

extern "C" {

// sorted[n]: sort_indexes(labels); buckets: the client buckets concatenated
// (positions into the sorted order), lens[num_clients] their sizes. Returns the
// number of buckets, or -1 when `cap` is too small / the set too small.
int fo_sampler_buckets(const int32_t* labels, int n, int num_clients, int outlier, int seed, int32_t* sorted,
                       int32_t* buckets, long cap, int32_t* lens) {
  std::srand((unsigned)seed);  // :387
  std::vector<int> train_labels(labels, labels + n);
  std::vector<size_t> indices = sort_indexes(train_labels);  // :416
  std::vector<int> range;
  for (int i = 0; i < n; i++) {
    sorted[i] = (int32_t)indices[(size_t)i];
    range.push_back(i);
  }
  std::vector<std::vector<int>> bks;
  int offset = 0, numOutliers = 0;
  if (outlier) {  // :427-443
    numOutliers = 1;
    while (offset < n && train_labels[indices[(size_t)offset]] == 0) offset++;
    std::vector<int> bucket;
    bucket.insert(bucket.end(), range.begin(), range.begin() + offset);
    std::random_shuffle(bucket.begin(), bucket.end(), [](int i) -> int { return std::rand() % i; });
    bks.push_back(bucket);
  }
  std::vector<int> shards;  // :446-449
  for (int i = 0; i < 2 * (num_clients - numOutliers); i++) shards.push_back(i);
  std::random_shuffle(shards.begin(), shards.end(), [](int i) -> int { return std::rand() % i; });
  int bucketSize = (int)(n - offset) / (num_clients - numOutliers);  // :452-453
  int shardSize = (int)bucketSize / 2;
  if (shardSize <= 0) return -1;
  for (size_t i = 0; i < shards.size(); i = i + 2) {  // :455-468
    std::vector<int> bucket;
    bucket.insert(bucket.end(), range.begin() + offset + shards[i] * shardSize,
                  range.begin() + offset + (shards[i] + 1) * shardSize);
    bucket.insert(bucket.end(), range.begin() + offset + shards[i + 1] * shardSize,
                  range.begin() + offset + (shards[i + 1] + 1) * shardSize);
    std::random_shuffle(bucket.begin(), bucket.end(), [](int i) -> int { return std::rand() % i; });
    bks.push_back(bucket);
  }
  long o = 0;
  for (size_t k = 0; k < bks.size(); ++k) {
    if (o + (long)bks[k].size() > cap) return -1;
    lens[k] = (int32_t)bks[k].size();
    for (int v : bks[k]) buckets[o++] = v;
  }
  return (int)bks.size();
}

}  // extern "C"
