// fleet_amd/csrc/sampler_state.cpp -- the offline sampler's state (fleet_sampler):
// what the reference's CppNNOfflineSampler natives keep in globals of
// libnative.so (Server/src/main/c++/cppNN_backend.cpp: train_images /
// train_labels, numLabels, iid / outlier / numClients, buckets / bucketIdx /
// sorted_images, currClientID, and E / sigma / C set by initUpdater), on top of
// the public C-ABI (fleet_codec.h: the mini-batch encode runs on the GPU).
//
//   fleet_sampler_create    initSampler (:385-479): srand(seed), the MNIST
//                           training set (commonLib/cppNN/mnist_parser.h), the
//                           non-IID buckets
//   fleet_updater_reseed(_ex) initUpdater's srand(seed) (:163) and the rand()
//                           draws of its one cnn.train_class (:216/:222) after a fetch
//   fleet_sampler_set_hyper initUpdater's E, sigma, C (:169-171)
//   fleet_sampler_minibatch getMiniBatch (:677-699) = uniformSample (:553-634)
//                           / nonIIDSample (:636-675) + Base64::encode
//
// Random numbers come from libc rand(), the process-wide generator the
// reference draws from; the shuffles are libstdc++'s std::random_shuffle
// algorithm over it (restated below; oracle/sampler_oracle.cpp runs the real
// one) and the label sort is the same std::sort call as sort_indexes (:116-127).
#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/fleet_codec.h"

struct fleet_sampler {
  fleet_ctx* ctx = nullptr;
  std::mutex mu;
  std::string err;
  int F = 0, num_labels = 0, iid = 0, outlier = 0, num_clients = 10, mode = 1, seed = 1;
  std::vector<float> images;        // train_images, n x F, as loaded
  std::vector<int32_t> labels;      // train_labels
  std::vector<int32_t> sorted_idx;  // sort_indexes(train_labels): sorted_images[i] = images[sorted_idx[i]]
  std::vector<std::vector<int32_t>> buckets;  // into the sorted order
  std::vector<size_t> bucket_pos;             // bucketIdx
  int curr_client = 0;                        // currClientID
  int E = 0;                                  // initUpdater's globals (zero until it runs)
  double sigma = 0.0, C = 0.0;
  std::vector<float> teacher_w, teacher_b;    // DISTILLATION_MODE=1 + iid: the trained teacher
  std::vector<int32_t> last_idx;              // the last request's images (loaded order)
  std::vector<int32_t> gather_idx;            // scratch
  std::vector<float> probs;                   // scratch
};

namespace {

int sfail(fleet_sampler* s, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (s) s->err = buf;
  return code;
}

// libstdc++'s std::random_shuffle(first, last, gen) (bits/stl_algo.h): for
// i = 1 .. n-1, j = gen(i + 1), swap(a[i], a[j]) when i != j -- with the
// reference's generator [](int i) { return std::rand() % i; } (:434, :449, :464)
void random_shuffle_rand(std::vector<int32_t>& a) {
  if (a.empty()) return;
  for (size_t i = 1; i < a.size(); ++i) {
    const size_t j = (size_t)(std::rand() % (int)(i + 1));
    if (i != j) std::swap(a[i], a[j]);
  }
}

uint32_t be32(const unsigned char* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

bool read_file(const std::string& path, std::vector<unsigned char>* out) {
  std::ifstream f(path, std::ios::in | std::ios::binary);
  if (!f) return false;
  out->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}

// mnist::parse_mnist_images / parse_mnist_labels (mnist_parser.h) with the
// defaults parse_train_data passes: pixels (b / 255.0f) * (1 - (-1)) + (-1), no
// padding; "<path>/train-images.idx3-ubyte", else "<path>/train-images-idx3-ubyte".
int load_mnist(fleet_sampler* s, const std::string& path, std::vector<float>* images, std::vector<int32_t>* labels) {
  std::vector<unsigned char> im, lb;
  if (!read_file(path + "/train-images.idx3-ubyte", &im) && !read_file(path + "/train-images-idx3-ubyte", &im))
    return sfail(s, FLEET_ERR_ARG, "could not parse data: no train-images idx3 file under %s", path.c_str());
  if (!read_file(path + "/train-labels.idx1-ubyte", &lb) && !read_file(path + "/train-labels-idx1-ubyte", &lb))
    return sfail(s, FLEET_ERR_ARG, "could not parse data: no train-labels idx1 file under %s", path.c_str());
  if (im.size() < 16 || lb.size() < 8) return sfail(s, FLEET_ERR_ARG, "truncated MNIST header");
  const uint32_t n = be32(&im[4]), rows = be32(&im[8]), cols = be32(&im[12]), nl = be32(&lb[4]);
  const size_t F = (size_t)rows * cols;
  if (F == 0 || F > (1u << 20) || im.size() < 16 + (size_t)n * F || lb.size() < 8 + (size_t)nl || nl != n)
    return sfail(s, FLEET_ERR_ARG, "MNIST files disagree or are truncated (%u images of %zu pixels, %u labels)", n,
                 F, nl);
  images->resize((size_t)n * F);
  labels->resize(n);
  const float scale_min = -1.0f, scale_max = 1.0f;
  for (size_t i = 0; i < (size_t)n * F; ++i)
    (*images)[i] = ((float)im[16 + i] / 255.0f) * (scale_max - scale_min) + scale_min;
  for (uint32_t i = 0; i < n; ++i) (*labels)[i] = lb[8 + i];
  s->F = (int)F;
  return FLEET_OK;
}

// initSampler after the dataset is loaded (:387, :401, :411-479): srand(seed),
// numLabels, and for the non-IID sampler the label sort and the buckets.
int build_state(fleet_sampler* s) {
  const size_t n = s->labels.size();
  if (n == 0) return sfail(s, FLEET_ERR_ARG, "empty dataset");
  std::srand((unsigned)s->seed);
  s->curr_client = 0;
  s->buckets.clear();
  s->bucket_pos.clear();
  s->sorted_idx.clear();
  if (s->iid) return FLEET_OK;
  // sort_indexes (:116-127): the same std::sort call (size_t indices, label compare)
  std::vector<size_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  const std::vector<int32_t>& v = s->labels;
  std::sort(idx.begin(), idx.end(), [&v](size_t i1, size_t i2) { return v[i1] < v[i2]; });
  s->sorted_idx.assign(idx.begin(), idx.end());
  size_t offset = 0;
  int num_outliers = 0;
  if (s->outlier) {  // the bucket of the label-0 samples (:427-443)
    num_outliers = 1;
    while (offset < n && v[idx[offset]] == 0) offset++;
    if (offset == n) return sfail(s, FLEET_ERR_ARG, "every sample has label 0: no non-outlier shards");
    std::vector<int32_t> bucket(offset);
    std::iota(bucket.begin(), bucket.end(), 0);
    random_shuffle_rand(bucket);
    s->buckets.push_back(bucket);
  }
  const int shards_n = 2 * (s->num_clients - num_outliers);
  if (shards_n <= 0) return sfail(s, FLEET_ERR_ARG, "numClients %d leaves no non-outlier client", s->num_clients);
  std::vector<int32_t> shards((size_t)shards_n);
  std::iota(shards.begin(), shards.end(), 0);
  random_shuffle_rand(shards);
  const int bucket_size = (int)(n - offset) / (s->num_clients - num_outliers);
  const int shard_size = bucket_size / 2;
  if (shard_size <= 0) return sfail(s, FLEET_ERR_ARG, "%zu samples are too few for %d clients", n, s->num_clients);
  for (size_t i = 0; i < shards.size(); i += 2) {  // two shards per client (:455-468)
    std::vector<int32_t> bucket;
    for (int sh : {shards[i], shards[i + 1]})
      for (int k = 0; k < shard_size; ++k) bucket.push_back((int32_t)offset + sh * shard_size + k);
    random_shuffle_rand(bucket);
    s->buckets.push_back(bucket);
  }
  s->bucket_pos.assign(s->buckets.size(), 0);
  return FLEET_OK;
}

int create_common(fleet_sampler* s, fleet_sampler** out) {
  const int rc = build_state(s);
  if (rc != FLEET_OK) {
    std::fprintf(stderr, "[fleet] initSampler: %s\n", s->err.c_str());
    delete s;
    return rc;
  }
  *out = s;
  return FLEET_OK;
}

}  // namespace

extern "C" {

int fleet_sampler_create(fleet_ctx* ctx, const char* data_path, int iid, int outlier, int num_clients,
                         int distillation_mode, int seed, fleet_sampler** out) {
  if (!data_path || !out || num_clients <= 0) return FLEET_ERR_ARG;
  *out = nullptr;
  fleet_sampler* s = new fleet_sampler();
  s->ctx = ctx;
  s->iid = iid != 0;
  s->outlier = outlier != 0;
  s->num_clients = num_clients;
  s->mode = distillation_mode != 0;
  s->seed = seed;
  s->num_labels = 10;  // MNIST (:401)
  int rc = load_mnist(s, data_path, &s->images, &s->labels);
  if (rc != FLEET_OK) {
    std::fprintf(stderr, "[fleet] initSampler: %s\n", s->err.c_str());
    delete s;
    return rc;
  }
  return create_common(s, out);
}

int fleet_sampler_create_from(fleet_ctx* ctx, const float* images, const int32_t* labels, size_t n, int F,
                              int num_labels, int iid, int outlier, int num_clients, int distillation_mode, int seed,
                              fleet_sampler** out) {
  if (!out || (n && (!images || !labels)) || F <= 0 || num_clients <= 0 || num_labels <= 0)
    return FLEET_ERR_ARG;
  *out = nullptr;
  fleet_sampler* s = new fleet_sampler();
  s->ctx = ctx;
  s->iid = iid != 0;
  s->outlier = outlier != 0;
  s->num_clients = num_clients;
  s->mode = distillation_mode != 0;
  s->seed = seed;
  s->num_labels = num_labels;
  s->F = F;
  s->images.assign(images, images + n * (size_t)F);
  s->labels.assign(labels, labels + n);
  return create_common(s, out);
}

void fleet_sampler_destroy(fleet_sampler* s) { delete s; }

const char* fleet_sampler_last_error(const fleet_sampler* s) { return s ? s->err.c_str() : "no sampler"; }

void fleet_updater_reseed_ex(int seed, int fetched) {
  std::srand((unsigned)seed);
  // cnn.train_class(train_images[0], ...) after it: the random shift of
  // set_random_augmentation(1, 1, 0, 0, edge) (fetchParamsNative :293) draws
  // rand() twice (network.h:1840; no flips, no OpenCV transform, no dropout in
  // the reference's MNIST network). Without a fetched model use_augmentation is 0.
  if (fetched) {
    (void)std::rand();
    (void)std::rand();
  }
}

void fleet_updater_reseed(int seed) { fleet_updater_reseed_ex(seed, 1); }

int fleet_sampler_set_hyper(fleet_sampler* s, int E, double sigma, double C) {
  if (!s) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(s->mu);
  s->E = E;
  s->sigma = sigma;
  s->C = C;
  return FLEET_OK;
}

int fleet_sampler_set_teacher(fleet_sampler* s, const float* w, size_t n_w, const float* b, size_t n_b) {
  if (!s || !w || !b || n_w != fleet_teacher_weight_count() || n_b != fleet_teacher_bias_count()) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(s->mu);
  if (s->F < 784) return sfail(s, FLEET_ERR_ARG, "the teacher takes 28x28 images, the set has %d features", s->F);
  s->teacher_w.assign(w, w + n_w);
  s->teacher_b.assign(b, b + n_b);
  return FLEET_OK;
}

size_t fleet_sampler_minibatch_len(fleet_sampler* s, int batch_size) {
  if (!s) return 0;
  std::lock_guard<std::mutex> lk(s->mu);
  const long B = (long)batch_size * s->E;
  if (B <= 0 || B > (1L << 24)) return 0;
  const bool teach = s->iid && s->mode;
  return fleet_minibatch_len(s->F, (int)B, s->num_labels, teach);
}

int fleet_sampler_minibatch(fleet_sampler* s, int batch_size, float lr, char* out, size_t cap, size_t* out_len) {
  if (!s) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(s->mu);
  if (!s->ctx) return sfail(s, FLEET_ERR_HIP, "no device context: the mini-batch encode runs on the GPU");
  const long B = (long)batch_size * s->E;  // batch_size *= E (:681)
  if (B <= 0 || B > (1L << 24))
    return sfail(s, FLEET_ERR_ARG,
                 "batch_size * E = %ld samples (E = %d: initUpdater not run?); the reference reads sample 0 of "
                 "an empty batch here",
                 B, s->E);
  const bool teach = s->iid && s->mode;  // uniformSample's DISTILLATION_MODE branch (:593-620)
  if (teach && s->teacher_w.empty())
    return sfail(s, FLEET_ERR_ARG,
                 "DISTILLATION_MODE=1 with iid sampling needs the trained teacher (initSampler :480-546 is not "
                 "rebuilt; fleet_sampler_set_teacher)");
  const size_t len = fleet_minibatch_len(s->F, (int)B, s->num_labels, teach);
  if (out_len) *out_len = len;
  if (!out || cap < len) return sfail(s, FLEET_ERR_CAPACITY, "output capacity %zu < %zu", cap, len);
  const size_t n = s->labels.size();
  s->gather_idx.resize((size_t)B);
  if (s->iid) {  // uniformSample (:559-566): index = 0 + rand() % (N - 1 - 0 + 1)
    for (long j = 0; j < B; ++j) s->gather_idx[(size_t)j] = (int32_t)(std::rand() % (int)n);
  } else {  // nonIIDSample (:645-652): the client's bucket, non-overlapping, wrapping around
    const int c = s->curr_client;
    if (c < 0 || (size_t)c >= s->buckets.size() || s->buckets[(size_t)c].empty())
      return sfail(s, FLEET_ERR_ARG, "client %d has no bucket", c);
    const std::vector<int32_t>& bk = s->buckets[(size_t)c];
    size_t& pos = s->bucket_pos[(size_t)c];
    for (long j = 0; j < B; ++j) {
      s->gather_idx[(size_t)j] = s->sorted_idx[(size_t)bk[pos]];
      pos = (pos + 1) % bk.size();
    }
  }
  s->curr_client = (s->curr_client + 1) % s->num_clients;  // :687
  // the header as push_back converts it (:585-591 / :655-661)
  const float header[7] = {(float)s->E, (float)s->sigma, (float)s->C, lr, (float)B, (float)s->F,
                           (float)s->num_labels};
  const float* teacher = nullptr;
  if (teach) {
    s->probs.resize((size_t)B * 10);
    const int rc = fleet_teacher_forward(s->ctx, s->teacher_w.data(), s->teacher_w.size(), s->teacher_b.data(),
                                         s->teacher_b.size(), s->images.data(), n, s->F, s->gather_idx.data(), (int)B,
                                         2.0f /* TEMPERATURE, network.h:53 */, s->probs.data());
    if (rc != FLEET_OK) return sfail(s, rc, "teacher forward: %s", fleet_last_error(s->ctx));
    teacher = s->probs.data();
  }
  const int rc = fleet_minibatch(s->ctx, s->images.data(), n, s->F, s->labels.data(), s->gather_idx.data(), (int)B,
                                 teacher, s->num_labels, header, out, cap, out_len);
  if (rc != FLEET_OK) return sfail(s, rc, "mini-batch encode: %s", fleet_last_error(s->ctx));
  s->last_idx = s->gather_idx;
  return FLEET_OK;
}

int fleet_sampler_num_labels(const fleet_sampler* s) { return s ? s->num_labels : 0; }
int fleet_sampler_has_outlier(const fleet_sampler* s) { return s ? s->outlier : 0; }
size_t fleet_sampler_num_samples(const fleet_sampler* s) { return s ? s->labels.size() : 0; }

int fleet_sampler_bucket(fleet_sampler* s, int client, int32_t* out, size_t cap, size_t* n) {
  if (!s || !n) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(s->mu);
  if (client < 0 || (size_t)client >= s->buckets.size()) return sfail(s, FLEET_ERR_ARG, "no bucket %d", client);
  const std::vector<int32_t>& b = s->buckets[(size_t)client];
  *n = b.size();
  if (cap < b.size() || (!out && !b.empty())) return FLEET_ERR_CAPACITY;
  std::copy(b.begin(), b.end(), out);
  return FLEET_OK;
}

int fleet_sampler_sorted_index(fleet_sampler* s, int32_t* out, size_t cap, size_t* n) {
  if (!s || !n) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(s->mu);
  *n = s->sorted_idx.size();
  if (cap < s->sorted_idx.size() || (!out && *n)) return FLEET_ERR_CAPACITY;
  std::copy(s->sorted_idx.begin(), s->sorted_idx.end(), out);
  return FLEET_OK;
}

int fleet_sampler_last_indices(fleet_sampler* s, int32_t* out, size_t cap, size_t* n) {
  if (!s || !n) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(s->mu);
  *n = s->last_idx.size();
  if (cap < s->last_idx.size() || (!out && *n)) return FLEET_ERR_CAPACITY;
  std::copy(s->last_idx.begin(), s->last_idx.end(), out);
  return FLEET_OK;
}

}  // extern "C"
