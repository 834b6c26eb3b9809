// Flat C ABI of the bf16 full-AlexNet engine (anx/c_api.h, "full AlexNet bf16 engine"): libanx_bf16.so.
// Its own library so the fp32 programs (the anx CLI, the Blocks engine) never load the bf16 kernels'
// code objects: the V3 process's cold start pays only for what it runs. Errors go through libanx's
// thread-local message (anx_set_last_error / anx_last_error).
#include <exception>
#include <stdexcept>
#include <string>

#include "anx/bf16_ops.hpp"
#include "anx/c_api.h"
#include "anx/knobs.hpp"

namespace {
int fail(const std::string& m) {
  anx_set_last_error(m.c_str());
  return 1;
}
int hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  return fail(std::string(what) + ": " + hipGetErrorString(e));
}
template <class F>
int guarded(const char* what, F&& f) {
  try {
    return f();
  } catch (const std::exception& ex) {
    return fail(std::string(what) + ": " + ex.what());
  } catch (...) {
    return fail(std::string(what) + ": unknown exception");
  }
}
hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }
}  // namespace

extern "C" {

int anx_full_weight_sizes(int classes, int groups2, size_t* wn, size_t* bn) {
  anx::full_weight_shapes(classes, groups2, wn, bn);
  return 0;
}

int anx_full_create(void** out, const float* const* weights, const float* const* biases, int classes,
                    int max_batch, int groups2, int lrn_mode) {
  return guarded("anx_full_create", [&] {
    size_t wn[8], bn[8];
    anx::full_weight_shapes(classes, groups2, wn, bn);
    anx::FullWeights w;
    for (int i = 0; i < 8; ++i) {
      w.w[i].assign(weights[i], weights[i] + wn[i]);
      w.b[i].assign(biases[i], biases[i] + bn[i]);
    }
    *out = new anx::FullEngine(w, classes, max_batch, groups2, static_cast<anx::LrnMode>(lrn_mode));
    return 0;
  });
}

int anx_full_destroy(void* e) {
  delete static_cast<anx::FullEngine*>(e);
  return 0;
}

int anx_full_forward(void* e, const float* x, int N, float* logits, void* stream) {
  return guarded("anx_full_forward", [&] {
    return hip_status(static_cast<anx::FullEngine*>(e)->forward(x, N, logits, S(stream)), "full forward");
  });
}

int anx_full_forward_mark(void* e, const float* x, int N, float* logits, void* stream) {
  return guarded("anx_full_forward_mark", [&] {
    return hip_status(static_cast<anx::FullEngine*>(e)->forward(x, N, logits, S(stream), true), "full forward");
  });
}

int anx_full_wait_mark(void* e, void* stream) {
  return guarded("anx_full_wait_mark", [&] {
    return hip_status(static_cast<anx::FullEngine*>(e)->wait_mark(S(stream)), "full wait mark");
  });
}

int anx_full_tap(void* e, int i, int N, void* dst, size_t* elems, void* stream) {
  *elems = static_cast<anx::FullEngine*>(e)->tap(i, N, dst, S(stream));
  return *elems ? 0 : fail("anx_full_tap: bad tap index or batch");
}
int anx_full_set_knob(void* e, const char* name, int value) {
  if (anx::set_knob(static_cast<anx::FullEngine*>(e)->knobs(), name, value) != 0)
    return fail(std::string("bad knob or value: ") + (name ? name : "(null)"));
  return 0;
}
int anx_full_get_knob(void* e, const char* name, int* value) {
  if (anx::get_knob(static_cast<anx::FullEngine*>(e)->knobs(), name, value) != 0)
    return fail(std::string("unknown knob: ") + (name ? name : "(null)"));
  return 0;
}
}  // extern "C"
