/*
 * oracle/ref_model_driver.cpp -- TEST INFRASTRUCTURE ONLY (oracle harness).
 *
 * Drives the reference's OWN DISTILLATION_MODE=1 model codec -- the header-only
 * mojo network of commonLib/cppNN compiled by path from /root/reference (see
 * oracle/Makefile) -- and exposes a flat C API for ctypes (tests, fixtures).
 * Nothing in fleet_amd/ links or loads this.
 *
 *   ref_quantize_params: an empty mojo::network whose W holds the given
 *     matrices; getParametersNative's mode-1 sequence on it
 *     (Server/src/main/c++/cppNN_backend.cpp:244-280: save_model_weights,
 *     quantization_weight_model, getParams, load_model_weights).
 *   ref_mnist_roundtrip: the Driver's MNIST network (Driver/src/main/c++/
 *     cppNN_backend.cpp:109-117) with its own weight init, optionally
 *     overwritten; the same mode-1 getParams, then network::read of that text
 *     into a fresh network (the client/Driver side, network.h:840-997).
 *   ref_server_session: the server's model natives replayed on a network read
 *     from a getParams text (fetchParamsNative, initUpdater, descentNative,
 *     getParametersNative, getModelParametersNative; cppNN_backend.cpp:161-383).
 *   ref_teacher_forward: the sampler's mode-1 teacher (initSampler's network,
 *     cppNN_backend.cpp:494-502) with the given W / biases, and uniformSample's
 *     teacher.forward(sample, TEMPERATURE, -1, 1) per sample (:603).
 */
#include <cstdio>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "mojo.h"

namespace {

size_t copy_out(const std::string& s, char* out, size_t cap) {
  if (out && cap) std::memcpy(out, s.data(), s.size() < cap ? s.size() : cap);
  return s.size();
}

std::string quantized_params(mojo::network& net) {
  std::vector<mojo::matrix*> unquantized;
  net.save_model_weights(&unquantized);
  net.quantization_weight_model();
  return net.getParams();
}

}  // namespace

extern "C" {

// dims: n_mats x {cols, rows, chans}; w: the concatenated matrices.
// wq_out (nullable): the quantised weights; returns the getParams text length.
size_t ref_quantize_params(const float* w, const int* dims, int n_mats, float* wq_out, char* text, size_t cap) {
  mojo::network net("sgd");
  size_t off = 0;
  for (int j = 0; j < n_mats; ++j) {
    mojo::matrix* m = new mojo::matrix(dims[3 * j], dims[3 * j + 1], dims[3 * j + 2]);
    std::memcpy(m->x, w + off, sizeof(float) * m->size());
    off += m->size();
    net.W.push_back(m);
  }
  std::vector<mojo::matrix*> unquantized;
  net.save_model_weights(&unquantized);
  net.quantization_weight_model();
  const std::string params = net.getParams();
  if (wq_out) {
    size_t o = 0;
    for (auto* m : net.W) {
      std::memcpy(wq_out + o, m->x, sizeof(float) * m->size());
      o += m->size();
    }
  }
  net.load_model_weights(unquantized);
  return copy_out(params, text, cap);
}

// The MNIST network. n_mats/dims_out (<= 16 matrices) describe its non-null W
// in order; w_in (nullable) overwrites the initial weights; w_init_out,
// wq_out, w_read_out (nullable) receive the initial, quantised and read-back
// weights. Returns the text length (call with text == NULL to size it).
size_t ref_mnist_roundtrip(const float* w_in, int* n_mats, int* dims_out, float* w_init_out, float* wq_out,
                           float* w_read_out, char* text, size_t cap) {
  mojo::network cnn("sgd");
  cnn.push_back("I1", "input 28 28 1");
  cnn.push_back("C1", "convolution 5 8 1 elu");
  cnn.push_back("P1", "semi_stochastic_pool 3 3");
  cnn.push_back("C2i", "convolution 1 16 1 elu");
  cnn.push_back("C2", "convolution 5 48 1 elu");
  cnn.push_back("P2", "semi_stochastic_pool 2 2");
  cnn.push_back("FC2", "softmax 10");
  cnn.connect_all();
  int nm = 0;
  size_t off = 0;
  for (auto* m : cnn.W) {
    if (!m) continue;
    if (dims_out) {
      dims_out[3 * nm] = m->cols;
      dims_out[3 * nm + 1] = m->rows;
      dims_out[3 * nm + 2] = m->chans;
    }
    if (w_in) std::memcpy(m->x, w_in + off, sizeof(float) * m->size());
    if (w_init_out) std::memcpy(w_init_out + off, m->x, sizeof(float) * m->size());
    off += m->size();
    ++nm;
  }
  if (n_mats) *n_mats = nm;
  std::vector<mojo::matrix*> unquantized;
  cnn.save_model_weights(&unquantized);
  cnn.quantization_weight_model();
  const std::string params = cnn.getParams();
  if (wq_out) {
    size_t o = 0;
    for (auto* m : cnn.W)
      if (m) {
        std::memcpy(wq_out + o, m->x, sizeof(float) * m->size());
        o += m->size();
      }
  }
  cnn.load_model_weights(unquantized);
  if (w_read_out) {
    mojo::network rd("sgd");
    std::istringstream ss(params);
    rd.read(ss);
    size_t o = 0;
    for (auto* m : rd.W)
      if (m) {
        std::memcpy(w_read_out + o, m->x, sizeof(float) * m->size());
        o += m->size();
      }
  }
  return copy_out(params, text, cap);
}

// descentNative's model step on the Driver's MNIST network
// (Server/src/main/c++/cppNN_backend.cpp:336-352: set_learning_rate, then
// network::descent(vector), network.h:1185-1202 -> :1334-1353 -> sgd
// solver.h:88-94 and fully_connected_layer::update_bias layer.h:241-243).
// One train_class on a blank image first sizes dW_sets/dbias_sets, as
// initUpdater does (:216-222). w_in (nullable) overwrites the non-null W in
// order; b_in (nullable) the biases of every layer with use_bias(), in layer
// order. Outputs (nullable): the gradients() layout sizes (w_sizes[n_w],
// b_sizes[n_b]), the W and biases before (w0, b0) and after (w1, b1) the
// step, and per layer fc[k] = (is a fully_connected_layer) | (bias size if
// use_bias(), else 0) << 1.
// g = the merged gradient (decodeFloat of mergeFlatGradient's output).
int ref_mnist_descent(const float* w_in, const float* b_in, const float* g, int n_g, float lr, int* n_w,
                      int* w_sizes, int* n_b, int* b_sizes, float* w0, float* b0, float* w1, float* b1, int* fc) {
  mojo::network cnn("sgd");
  cnn.push_back("I1", "input 28 28 1");
  cnn.push_back("C1", "convolution 5 8 1 elu");
  cnn.push_back("P1", "semi_stochastic_pool 3 3");
  cnn.push_back("C2i", "convolution 1 16 1 elu");
  cnn.push_back("C2", "convolution 5 48 1 elu");
  cnn.push_back("P2", "semi_stochastic_pool 2 2");
  cnn.push_back("FC2", "softmax 10");
  cnn.connect_all();
  cnn.start_epoch("cross_entropy");
  std::vector<float> blank(28 * 28, 0.0f);
  cnn.train_class(blank.data(), 3, NULL);
  auto& layers = cnn.layer_sets[mojo::network::MAIN_LAYER_SET];
  auto copy_w = [&](float* dst, const float* src) {
    size_t o = 0;
    for (auto* m : cnn.W)
      if (m) {
        if (src) std::memcpy(m->x, src + o, sizeof(float) * m->size());
        if (dst) std::memcpy(dst + o, m->x, sizeof(float) * m->size());
        o += m->size();
      }
  };
  auto copy_b = [&](float* dst, const float* src) {
    size_t o = 0;
    for (auto* l : layers)
      if (l->use_bias()) {
        if (src) std::memcpy(l->bias.x, src + o, sizeof(float) * l->bias.size());
        if (dst) std::memcpy(dst + o, l->bias.x, sizeof(float) * l->bias.size());
        o += l->bias.size();
      }
  };
  copy_w(w0, w_in);
  copy_b(b0, b_in);
  if (n_w) *n_w = (int)cnn.dW_sets[0].size();
  if (w_sizes)
    for (size_t i = 0; i < cnn.dW_sets[0].size(); ++i) w_sizes[i] = cnn.dW_sets[0][i].size();
  if (n_b) *n_b = (int)cnn.dbias_sets[0].size();
  if (b_sizes)
    for (size_t i = 0; i < cnn.dbias_sets[0].size(); ++i) b_sizes[i] = cnn.dbias_sets[0][i].size();
  if (fc)
    for (size_t k = 0; k < layers.size(); ++k)
      fc[k] = (dynamic_cast<mojo::fully_connected_layer*>(layers[k]) != NULL) |
              ((layers[k]->use_bias() ? (int)layers[k]->bias.size() : 0) << 1);
  if (!g) return (int)layers.size();
  cnn.set_learning_rate(lr);
  cnn.descent(std::vector<float>(g, g + n_g));
  copy_w(w1, NULL);
  copy_b(b1, NULL);
  return (int)layers.size();
}

// getModelParametersNative's vector (Server/src/main/c++/cppNN_backend.cpp:
// 227-242 -> network::getModelParams, commonLib/cppNN/network.h:708-723) of the
// Driver's MNIST network, optionally with its W / use_bias() biases overwritten
// (w_in, b_in as in ref_mnist_descent). Returns the vector length; out nullable.
// (The bias loop sits inside a loop over layer_graph, so the biases repeat
// layer_graph.size() times before the weights.)
int ref_mnist_model_params(const float* w_in, const float* b_in, float* out, int* graph_edges) {
  mojo::network cnn("sgd");
  cnn.push_back("I1", "input 28 28 1");
  cnn.push_back("C1", "convolution 5 8 1 elu");
  cnn.push_back("P1", "semi_stochastic_pool 3 3");
  cnn.push_back("C2i", "convolution 1 16 1 elu");
  cnn.push_back("C2", "convolution 5 48 1 elu");
  cnn.push_back("P2", "semi_stochastic_pool 2 2");
  cnn.push_back("FC2", "softmax 10");
  cnn.connect_all();
  size_t o = 0;
  for (auto* m : cnn.W)
    if (m) {
      if (w_in) std::memcpy(m->x, w_in + o, sizeof(float) * m->size());
      o += m->size();
    }
  o = 0;
  for (auto* l : cnn.layer_sets[mojo::network::MAIN_LAYER_SET])
    if (l->use_bias()) {
      if (b_in) std::memcpy(l->bias.x, b_in + o, sizeof(float) * l->bias.size());
      o += l->bias.size();
    }
  const std::vector<float> v = cnn.getModelParams();
  if (out) std::memcpy(out, v.data(), sizeof(float) * v.size());
  if (graph_edges) *graph_edges = (int)cnn.layer_graph.size();
  return (int)v.size();
}

// descentNative's model copy (Server/src/main/c++/cppNN_backend.cpp:355-372):
// a fresh network reads the MNIST network's getParams() text (unquantised, mode 1).
void ref_mnist_version_copy(const float* w_in, const float* b_in, float* w_out, float* b_out) {
  mojo::network cnn("sgd");
  cnn.push_back("I1", "input 28 28 1");
  cnn.push_back("C1", "convolution 5 8 1 elu");
  cnn.push_back("P1", "semi_stochastic_pool 3 3");
  cnn.push_back("C2i", "convolution 1 16 1 elu");
  cnn.push_back("C2", "convolution 5 48 1 elu");
  cnn.push_back("P2", "semi_stochastic_pool 2 2");
  cnn.push_back("FC2", "softmax 10");
  cnn.connect_all();
  size_t o = 0;
  for (auto* m : cnn.W)
    if (m) {
      if (w_in) std::memcpy(m->x, w_in + o, sizeof(float) * m->size());
      o += m->size();
    }
  o = 0;
  for (auto* l : cnn.layer_sets[mojo::network::MAIN_LAYER_SET])
    if (l->use_bias()) {
      if (b_in) std::memcpy(l->bias.x, b_in + o, sizeof(float) * l->bias.size());
      o += l->bias.size();
    }
  mojo::network cnew("sgd");
  std::istringstream ss(cnn.getParams());
  cnew.read(ss);
  o = 0;
  for (auto* m : cnew.W)
    if (m) {
      std::memcpy(w_out + o, m->x, sizeof(float) * m->size());
      o += m->size();
    }
  o = 0;
  for (auto* l : cnew.layer_sets[mojo::network::MAIN_LAYER_SET])
    if (l->use_bias()) {
      std::memcpy(b_out + o, l->bias.x, sizeof(float) * l->bias.size());
      o += l->bias.size();
    }
}

// The updater's model natives of Server/src/main/c++/cppNN_backend.cpp replayed
// on the reference's own network code (DISTILLATION_MODE=1):
//   fetchParamsNative(text)          :282-301  cnn.read; start_epoch("distillation")
//   initUpdater(lrates)              :161-225  set_learning_rate(lrates[0]); models <- read(getParams());
//                                              one train_class (blank input, label 0, uniform
//                                              teacher probabilities) sizes dW_sets
//   descentNative(g_i, batch, stale) :329-383  set_mini_batch_size; lr = lrates[epoch] while
//                                              epoch < n; descent(g_i); epoch++; models <- read(getParams());
//                                              oldest dropped beyond stale
// g = n_steps merged gradients (decodeFloat of the merged Base64), n_g floats each.
// After init and after every step, the newest and the oldest version's
// getParametersNative text (save, quantize, getParams, restore) and getModelParams
// vector are appended to `out` as records {u64 n, bytes} / {u64 n, floats}, then
// models.size() as a u64. Returns the bytes needed (call with out == NULL to size it).
size_t ref_server_session(const char* text, size_t len, const double* lrates, int n_lr, const float* g, int n_g,
                          int n_steps, int batch, int stale, char* out, size_t cap) {
  std::string buf;
  auto put_text = [&](const std::string& t) {
    const uint64_t n = t.size();
    buf.append(reinterpret_cast<const char*>(&n), 8);
    buf += t;
  };
  auto put_floats = [&](const std::vector<float>& v) {
    const uint64_t n = v.size();
    buf.append(reinterpret_cast<const char*>(&n), 8);
    buf.append(reinterpret_cast<const char*>(v.data()), sizeof(float) * v.size());
  };
  auto quantized_text = [](mojo::network* net) {
    std::vector<mojo::matrix*> unq;
    net->save_model_weights(&unq);
    net->quantization_weight_model();
    const std::string t = net->getParams();
    net->load_model_weights(unq);
    return t;
  };
  mojo::network cnn("sgd");
  {
    std::istringstream ss(std::string(text, len));
    cnn.start_epoch("distillation");
    cnn.set_random_augmentation(1, 1, 0, 0, mojo::edge);
    cnn.clear();
    cnn.read(ss);
  }
  std::vector<mojo::network*> models;
  auto push_version = [&]() {
    mojo::network* nw = new mojo::network("sgd");
    nw->start_epoch("distillation");
    nw->set_random_augmentation(1, 1, 0, 0, mojo::edge);
    std::istringstream ss(cnn.getParams());
    nw->clear();
    nw->read(ss);
    models.push_back(nw);
  };
  auto record = [&]() {
    for (mojo::network* v : {models.back(), models.front()}) {
      put_text(quantized_text(v));
      put_floats(v->getModelParams());
    }
  };
  cnn.set_learning_rate(lrates[0]);
  push_version();
  {
    auto& layers = cnn.layer_sets[mojo::network::MAIN_LAYER_SET];
    const mojo::matrix& in = layers.front()->node;
    std::vector<float> blank((size_t)in.cols * in.rows * in.chans, 0.0f);
    const int n_out = layers.back()->node.size();
    std::vector<float> teacher((size_t)n_out, 1.0f / (float)n_out);
    cnn.train_class(blank.data(), 0, &teacher);
  }
  record();
  int epoch = 0;
  for (int i = 0; i < n_steps; ++i) {
    cnn.set_mini_batch_size(batch);
    if (epoch < n_lr) cnn.set_learning_rate(lrates[epoch]);
    cnn.descent(std::vector<float>(g + (size_t)i * n_g, g + (size_t)(i + 1) * n_g));
    ++epoch;
    push_version();
    if ((int)models.size() > stale) {
      delete models.front();
      models.erase(models.begin());
    }
    record();
  }
  const uint64_t nm = models.size();
  buf.append(reinterpret_cast<const char*>(&nm), 8);
  for (auto* v : models) delete v;
  return copy_out(buf, out, cap);
}

}  // extern "C"

extern "C" {

// w: the teacher's non-null W in network order, b: the use_bias() layers' biases
// in layer order; x: B samples of 784 floats; probs: B x 10.
int ref_teacher_forward(const float* w, const float* b, const float* x, int B, float* probs) {
  mojo::network teacher("sgd");
  teacher.set_smart_training(false);
  teacher.set_learning_rate(0.01f);
  teacher.push_back("I1", "input 28 28 1");
  teacher.push_back("C1", "convolution 5 8 1 elu");
  teacher.push_back("P1", "semi_stochastic_pool 3 3");
  teacher.push_back("C2i", "convolution 1 16 1 elu");
  teacher.push_back("C2", "convolution 5 48 1 elu");
  teacher.push_back("P2", "semi_stochastic_pool 2 2");
  teacher.push_back("FC2", "softmax 10");
  teacher.connect_all();
  size_t o = 0;
  for (auto* m : teacher.W)
    if (m) {
      std::memcpy(m->x, w + o, sizeof(float) * m->size());
      o += m->size();
    }
  size_t ob = 0;
  for (auto* l : teacher.layer_sets[mojo::network::MAIN_LAYER_SET])
    if (l->use_bias()) {
      std::memcpy(l->bias.x, b + ob, sizeof(float) * l->bias.size());
      ob += l->bias.size();
    }
  for (int i = 0; i < B; ++i) {
    const float* out = teacher.forward(x + (size_t)i * 784, TEMPERATURE, -1, 1);
    std::memcpy(probs + (size_t)i * 10, out, sizeof(float) * 10);
  }
  return (int)(o * 1000 + ob);
}

}  // extern "C"

