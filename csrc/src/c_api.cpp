// Flat C ABI (see anx/c_api.h). Exceptions and HIP errors are converted to status codes +
// a thread-local message so nothing unwinds across the ctypes boundary.
#include "anx/c_api.h"

#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>
#include <vector>
#include <algorithm>

#include "anx/cost.hpp"
#include "anx/cpu_engine.hpp"
#include "anx/engine.hpp"
#include "anx/ops.hpp"
#include "anx/plan.hpp"
#include "anx/rng.hpp"

namespace {
thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
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

anx::BlockSpec from_c(const anx_block_c& b) {
  anx::BlockSpec s{};
  s.conv = {b.C, b.K, b.F, b.S, b.P, b.groups};
  s.pool = {b.pool_F, b.pool_S};
  s.has_lrn = b.has_lrn != 0;
  s.lrn = {b.lrn_N, b.lrn_alpha, b.lrn_beta, b.lrn_k, static_cast<anx::LrnMode>(b.lrn_mode)};
  return s;
}
anx_block_c to_c(const anx::BlockSpec& s) {
  anx_block_c b{};
  b.C = s.conv.C;
  b.K = s.conv.K;
  b.F = s.conv.F;
  b.S = s.conv.S;
  b.P = s.conv.P;
  b.groups = s.conv.groups;
  b.pool_F = s.pool.F;
  b.pool_S = s.pool.S;
  b.has_lrn = s.has_lrn ? 1 : 0;
  b.lrn_N = s.lrn.N;
  b.lrn_alpha = s.lrn.alpha;
  b.lrn_beta = s.lrn.beta;
  b.lrn_k = s.lrn.k;
  b.lrn_mode = static_cast<int>(s.lrn.mode);
  return b;
}
anx::TilePlan tile_from_c(const anx_tile_c& t) {
  anx::TilePlan p;
  p.in = {t.in_lo, t.in_hi};
  p.c1 = {t.c1_lo, t.c1_hi};
  p.p1 = {t.p1_lo, t.p1_hi};
  p.q = {t.q_lo, t.q_hi};
  p.c2 = {t.c2_lo, t.c2_hi};
  p.out = {t.out_lo, t.out_hi};
  return p;
}
anx_tile_c tile_to_c(const anx::TilePlan& p) {
  return {p.in.lo, p.in.hi, p.c1.lo, p.c1.hi, p.p1.lo, p.p1.hi, p.q.lo, p.q.hi, p.c2.lo, p.c2.hi, p.out.lo, p.out.hi};
}
hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }
}  // namespace

extern "C" void anx_set_last_error(const char* msg) { g_err = msg ? msg : ""; }

namespace {

// ConvPlan <-> 16 ints
void plan_to_ints(const anx::hip::ConvPlan& p, int* o) {
  const int v[16] = {p.N, p.Hp, p.Wp, p.C, p.K, p.F, p.S, p.groups, p.Ho, p.Wo, p.Cg, p.Kg, p.kdim, p.kpad, p.kpad_n,
                     p.variant | (p.vec4 << 8) | (p.taps4 << 9)};
  std::memcpy(o, v, sizeof v);
}
anx::hip::ConvPlan plan_from_ints(const int* o) {
  anx::hip::ConvPlan p{};
  p.N = o[0];
  p.Hp = o[1];
  p.Wp = o[2];
  p.C = o[3];
  p.K = o[4];
  p.F = o[5];
  p.S = o[6];
  p.groups = o[7];
  p.Ho = o[8];
  p.Wo = o[9];
  p.Cg = o[10];
  p.Kg = o[11];
  p.kdim = o[12];
  p.kpad = o[13];
  p.kpad_n = o[14];
  p.variant = o[15] & 0xff;
  p.vec4 = (o[15] >> 8) & 1;
  p.taps4 = (o[15] >> 9) & 1;
  return p;
}
}  // namespace

extern "C" {

const char* anx_last_error(void) { return g_err.c_str(); }
int anx_abi_version(void) { return 1; }

int anx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void anx_default_blocks(anx_block_c* b1, anx_block_c* b2) {
  *b1 = to_c(anx::kBlock1);
  *b2 = to_c(anx::kBlock2);
}

int anx_make_plan(int H, int W, int np, int mode, const anx_block_c* b1, const anx_block_c* b2, anx_tile_c* tiles,
                  int* owned_in, int* owned_p1, anx_xfer_c* in_halos, int* n_in_halos, anx_xfer_c* p1_halos,
                  int* n_p1_halos, int cap) {
  return guarded("anx_make_plan", [&] {
    if (np < 1) return fail("np must be >= 1");
    const anx::DecompPlan p = anx::make_plan(H, W, np, static_cast<anx::Decomp>(mode), from_c(*b1), from_c(*b2));
    const char* err = anx::check_plan(p);
    if (err[0]) return fail(err);
    for (int t = 0; t < np; ++t) {
      tiles[t] = tile_to_c(p.tiles[t]);
      owned_in[2 * t] = p.owned_in[t].lo;
      owned_in[2 * t + 1] = p.owned_in[t].hi;
      owned_p1[2 * t] = p.owned_p1[t].lo;
      owned_p1[2 * t + 1] = p.owned_p1[t].hi;
    }
    if (static_cast<int>(p.in_halos.size()) > cap || static_cast<int>(p.p1_halos.size()) > cap)
      return fail("halo list exceeds capacity");
    *n_in_halos = static_cast<int>(p.in_halos.size());
    for (size_t i = 0; i < p.in_halos.size(); ++i)
      in_halos[i] = {p.in_halos[i].src, p.in_halos[i].dst, p.in_halos[i].rows.lo, p.in_halos[i].rows.hi};
    *n_p1_halos = static_cast<int>(p.p1_halos.size());
    for (size_t i = 0; i < p.p1_halos.size(); ++i)
      p1_halos[i] = {p.p1_halos[i].src, p.p1_halos[i].dst, p.p1_halos[i].rows.lo, p.p1_halos[i].rows.hi};
    return 0;
  });
}

int anx_make_hybrid_plan(int H, int W, int np, int batch, int row_ways, int mode, const anx_block_c* b1,
                         const anx_block_c* b2, int* groups, int* group, int* index, int* img, int* gsize,
                         anx_tile_c* tile, double* redundancy) {
  return guarded("anx_make_hybrid_plan", [&] {
    anx::HybridPlan p;
    if (!anx::make_hybrid_plan(H, W, np, batch, row_ways, static_cast<anx::Decomp>(mode), p, from_c(*b1),
                               from_c(*b2)))
      return fail("invalid hybrid plan request (np >= 1, batch >= 1, row_ways dividing np)");
    for (int g = 0; g < p.groups; ++g) {
      const char* err = anx::check_plan(p.row_plans[g]);
      if (err[0]) return fail(err);
      gsize[g] = p.group_size[g];
    }
    *groups = p.groups;
    for (int r = 0; r < np; ++r) {
      group[r] = p.group_of[r];
      index[r] = p.index_in_group[r];
      img[2 * r] = p.images[p.group_of[r]].lo;
      img[2 * r + 1] = p.images[p.group_of[r]].hi;
      tile[r] = tile_to_c(p.tile(r));
    }
    *redundancy = anx::conv1_redundancy(p);
    return 0;
  });
}

int anx_engine_create(void** out, const anx_block_c* b1, const anx_block_c* b2, int H, int W, const float* w1,
                      const float* bias1, const float* w2, const float* bias2, int max_batch, int impl) {
  return guarded("anx_engine_create", [&] {
    const anx::BlockSpec s1 = from_c(*b1), s2 = from_c(*b2);
    anx::HostWeights hw;
    anx::init_const(hw, s1, s2);
    std::memcpy(hw.w1.data(), w1, hw.w1.size() * sizeof(float));
    std::memcpy(hw.b1.data(), bias1, hw.b1.size() * sizeof(float));
    std::memcpy(hw.w2.data(), w2, hw.w2.size() * sizeof(float));
    std::memcpy(hw.b2.data(), bias2, hw.b2.size() * sizeof(float));
    *out = new anx::BlocksEngine(s1, s2, H, W, hw, max_batch, static_cast<anx::Impl>(impl));
    return 0;
  });
}

int anx_engine_destroy(void* e) {
  delete static_cast<anx::BlocksEngine*>(e);
  return 0;
}

int anx_engine_forward(void* e, const float* x, int N, float* y, void* stream) {
  return guarded("anx_engine_forward", [&] {
    return hip_status(static_cast<anx::BlocksEngine*>(e)->forward(x, N, y, S(stream)), "engine forward");
  });
}

int anx_engine_tile_forward(void* e, const float* x, int N, const anx_tile_c* t, float* y, void* stream) {
  return guarded("anx_engine_tile_forward", [&] {
    return hip_status(static_cast<anx::BlocksEngine*>(e)->tile_forward(x, N, tile_from_c(*t), y, S(stream)),
                      "engine tile_forward");
  });
}

int anx_engine_stage1(void* e, const float* x, int N, const anx_tile_c* t, void* stream) {
  return guarded("anx_engine_stage1", [&] {
    return hip_status(static_cast<anx::BlocksEngine*>(e)->stage1(x, N, tile_from_c(*t), S(stream)), "engine stage1");
  });
}

int anx_engine_stage2(void* e, int N, const anx_tile_c* t, float* y, void* stream) {
  return guarded("anx_engine_stage2", [&] {
    return hip_status(static_cast<anx::BlocksEngine*>(e)->stage2(N, tile_from_c(*t), y, S(stream)), "engine stage2");
  });
}

int anx_engine_window(void* e, const anx_tile_c* t, int n, int r, float** ptr, size_t* row_floats,
                      size_t* image_floats) {
  auto* eng = static_cast<anx::BlocksEngine*>(e);
  const anx::TilePlan tp = tile_from_c(*t);
  *ptr = eng->q2_row_ptr(tp, n, r);
  *row_floats = eng->q2_row_floats();
  *image_floats = eng->q2_image_stride_floats(tp);
  return 0;
}


int anx_cpu_engine_create(void** out, const anx_block_c* b1, const anx_block_c* b2, int H, int W, const float* w1,
                          const float* bias1, const float* w2, const float* bias2) {
  return guarded("anx_cpu_engine_create", [&] {
    const anx::BlockSpec s1 = from_c(*b1), s2 = from_c(*b2);
    anx::HostWeights hw;
    anx::init_const(hw, s1, s2);
    std::memcpy(hw.w1.data(), w1, hw.w1.size() * sizeof(float));
    std::memcpy(hw.b1.data(), bias1, hw.b1.size() * sizeof(float));
    std::memcpy(hw.w2.data(), w2, hw.w2.size() * sizeof(float));
    std::memcpy(hw.b2.data(), bias2, hw.b2.size() * sizeof(float));
    *out = new anx::CpuBlocks(s1, s2, H, W, hw);
    return 0;
  });
}

int anx_cpu_engine_destroy(void* e) {
  delete static_cast<anx::CpuBlocks*>(e);
  return 0;
}

int anx_cpu_engine_tile_forward(void* e, const float* x, int N, const anx_tile_c* t, float* y) {
  return guarded("anx_cpu_engine_tile_forward", [&] {
    static_cast<anx::CpuBlocks*>(e)->tile_forward(x, N, tile_from_c(*t), y);
    return 0;
  });
}

int anx_cpu_engine_stage1(void* e, const float* x, int N, const anx_tile_c* t) {
  return guarded("anx_cpu_engine_stage1", [&] {
    static_cast<anx::CpuBlocks*>(e)->stage1(x, N, tile_from_c(*t));
    return 0;
  });
}

int anx_cpu_engine_stage2(void* e, int N, const anx_tile_c* t, float* y) {
  return guarded("anx_cpu_engine_stage2", [&] {
    static_cast<anx::CpuBlocks*>(e)->stage2(N, tile_from_c(*t), y);
    return 0;
  });
}

int anx_cpu_engine_window(void* e, const anx_tile_c* t, int n, int r, float** ptr, size_t* row_floats,
                          size_t* image_floats) {
  auto* eng = static_cast<anx::CpuBlocks*>(e);
  const anx::TilePlan tp = tile_from_c(*t);
  *ptr = eng->window_row(tp, n, r);
  *row_floats = eng->window_row_floats();
  *image_floats = static_cast<size_t>(tp.q.size()) * eng->window_row_floats();
  return 0;
}

int anx_memcpy2d_host(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes, size_t height) {
  for (size_t i = 0; i < height; ++i)
    std::memcpy(static_cast<char*>(dst) + i * dpitch, static_cast<const char*>(src) + i * spitch, width_bytes);
  return 0;
}

int anx_memcpy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes, size_t height,
                       void* stream) {
  return hip_status(hipMemcpy2DAsync(dst, dpitch, src, spitch, width_bytes, height, hipMemcpyDefault, S(stream)),
                    "hipMemcpy2DAsync");
}

int anx_conv2d_direct(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C, int K,
                      int F, int S_, int P, int groups, int relu, void* stream) {
  return hip_status(anx::hip::conv2d_direct(x, w, b, y, N, H, W, C, K, F, S_, P, groups, relu != 0, S(stream)),
                    "conv2d_direct");
}

int anx_relu(float* x, size_t n, void* stream) { return hip_status(anx::hip::relu(x, n, S(stream)), "relu"); }
int anx_channel_copy(void* dst, const void* src, size_t bytes, int workgroups, void* stream) {
  return hip_status(anx::hip::channel_copy(dst, src, bytes, workgroups, S(stream)), "channel_copy");
}

int anx_maxpool_direct(const float* x, float* y, int N, int H, int W, int C, int F, int S_, void* stream) {
  return hip_status(anx::hip::maxpool_direct(x, y, N, H, W, C, F, S_, S(stream)), "maxpool_direct");
}

int anx_lrn_direct(const float* x, float* y, int N, int H, int W, int C, int size, float alpha, float beta, float k,
                   int mode, void* stream) {
  return hip_status(anx::hip::lrn_direct(x, y, N, H, W, C, size, alpha, beta, k, static_cast<anx::LrnMode>(mode),
                                         S(stream)),
                    "lrn_direct");
}

int anx_maxpool(const float* x, int N, int H, int W, int C, int F, int S_, float* out, int Hb, int Wb, int Cb,
                int h_off, int w_off, int c_off, void* stream) {
  return hip_status(
      anx::hip::maxpool(x, N, H, W, C, F, S_, anx::hip::OutView{out, Hb, Wb, Cb, h_off, w_off, c_off}, S(stream)),
      "maxpool");
}

int anx_maxpool_lrn(const float* x, float* y, int N, int H, int W, int C, int F, int S_, int size, float alpha,
                    float beta, float k, int mode, void* stream) {
  return hip_status(anx::hip::maxpool_lrn(x, y, N, H, W, C, F, S_, size, alpha, beta, k,
                                          static_cast<anx::LrnMode>(mode), S(stream)),
                    "maxpool_lrn");
}

int anx_conv_plan(int N, int Hp, int Wp, int C, int K, int F, int S_, int groups, int* plan_out,
                  size_t* packed_floats, size_t* koff_ints) {
  return guarded("anx_conv_plan", [&] {
    if (groups < 1 || C % groups || K % groups) return fail("channels must divide by groups");
    const auto p = anx::hip::make_conv_plan(N, Hp, Wp, C, K, F, S_, groups);
    plan_to_ints(p, plan_out);
    *packed_floats = anx::hip::packed_weight_floats(p);
    *koff_ints = anx::hip::koff_ints(p);
    return 0;
  });
}

int anx_conv_pack(const int* plan, const float* w_kcff, float* packed, int* koff) {
  return guarded("anx_conv_pack", [&] {
    const auto p = plan_from_ints(plan);
    std::vector<float> pk;
    std::vector<int> ko;
    anx::hip::pack_conv_weights_host(p, w_kcff, pk, ko);
    std::memcpy(packed, pk.data(), pk.size() * sizeof(float));
    std::memcpy(koff, ko.data(), ko.size() * sizeof(int));
    return 0;
  });
}

int anx_engine_set_knob(void* e, const char* name, int value) {
  // set_knob may (re)build weights and workspace (prepare(): hipMalloc / uploads that throw on failure):
  // an exception must not cross the C ABI
  return guarded("anx_engine_set_knob", [&] {
    if (static_cast<anx::BlocksEngine*>(e)->set_knob(name, value) != 0)
      return fail(std::string("bad knob or value: ") + (name ? name : "(null)"));
    return 0;
  });
}
int anx_engine_get_knob(void* e, const char* name, int* value) {
  if (anx::get_knob(static_cast<anx::BlocksEngine*>(e)->knobs(), name, value) != 0)
    return fail(std::string("unknown knob: ") + (name ? name : "(null)"));
  return 0;
}
int anx_default_knob(const char* name, int* value) {
  if (anx::get_knob(anx::default_knobs(), name, value) != 0)
    return fail(std::string("unknown knob: ") + (name ? name : "(null)"));
  return 0;
}

int anx_conv1_wino(const float* x, int N, int Hin, int W, const float* w_kcff, int K, int F, const float* bias,
                   float* y, int relu, void* stream) {
  return guarded("anx_conv1_wino", [&] {
    if (!anx::hip::conv1_wino_eligible(3, K, F, 4, 0, 1)) return fail("anx_conv1_wino: shape not eligible");
    const auto w = anx::hip::make_conv1_wino_plan(N, Hin, W, K, F);
    std::vector<float> u;
    anx::hip::conv1_wino_weights_host(K, F, w_kcff, u);
    float *dv = nullptr, *du = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&dv), std::max<size_t>(anx::hip::conv1_wino_v_floats(w), 1) * 4) != hipSuccess)
      return fail("anx_conv1_wino: hipMalloc");
    if (hipMalloc(reinterpret_cast<void**>(&du), u.size() * 4) != hipSuccess) {
      (void)hipFree(dv);
      return fail("anx_conv1_wino: hipMalloc");
    }
    hipError_t e = hipMemcpy(du, u.data(), u.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = anx::hip::conv1_wino(w, x, dv, du, bias, anx::hip::OutView{y, w.H1, w.W1, K, 0, 0, 0}, relu != 0, S(stream),
                               anx::default_knobs());
    if (e == hipSuccess) e = hipStreamSynchronize(S(stream));  // the workspaces are freed below
    (void)hipFree(dv);
    (void)hipFree(du);
    return hip_status(e, "conv1_wino");
  });
}

int anx_conv2_wino_tile(const float* x, int N, int Hq, int Wq, int C, const float* w_kcff, int K, int groups,
                        const float* bias, float* y, int relu, void* stream, int m) {
  return guarded("anx_conv2_wino", [&] {
    if ((m != 3 && m != 4) || !anx::hip::wino_eligible(5, 1, C, K, groups, m))
      return fail("anx_conv2_wino: shape not eligible");
    const auto w = anx::hip::make_wino_plan(N, Hq, Wq, C, K, groups, m);
    std::vector<float> u;
    anx::hip::wino_transform_weights_host(w, w_kcff, u);
    float *dv = nullptr, *du = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&dv), std::max<size_t>(anx::hip::wino_v_floats(w), 1) * 4) != hipSuccess)
      return fail("anx_conv2_wino: hipMalloc");
    if (hipMalloc(reinterpret_cast<void**>(&du), u.size() * 4) != hipSuccess) {
      (void)hipFree(dv);
      return fail("anx_conv2_wino: hipMalloc");
    }
    hipError_t e = hipMemcpy(du, u.data(), u.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = anx::hip::wino_input(w, x, dv, S(stream));
    if (e == hipSuccess)
      e = anx::hip::wino_conv2(w, dv, du, bias, anx::hip::OutView{y, w.Ho, w.Wo, K, 0, 0, 0}, relu != 0, S(stream),
                               anx::default_knobs());
    if (e == hipSuccess) e = hipStreamSynchronize(S(stream));  // the workspaces are freed below
    (void)hipFree(dv);
    (void)hipFree(du);
    return hip_status(e, "conv2_wino");
  });
}

int anx_conv2_wino(const float* x, int N, int Hq, int Wq, int C, const float* w_kcff, int K, int groups,
                   const float* bias, float* y, int relu, void* stream) {
  return anx_conv2_wino_tile(x, N, Hq, Wq, C, w_kcff, K, groups, bias, y, relu, stream, 3);
}

int anx_conv2d_mfma(const int* plan, const float* x, const float* wpacked, const int* koff, const float* bias,
                    float* out, int Hb, int Wb, int Cb, int h_off, int w_off, int c_off, int relu, void* stream) {
  const auto p = plan_from_ints(plan);
  return hip_status(anx::hip::conv2d_mfma(p, x, wpacked, koff, bias,
                                          anx::hip::OutView{out, Hb, Wb, Cb, h_off, w_off, c_off}, relu != 0,
                                          S(stream)),
                    "conv2d_mfma");
}

int anx_cpu_conv2d(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C, int K, int F,
                   int S_, int P, int groups, int relu) {
  return guarded("anx_cpu_conv2d", [&] {
    anx::cpu::conv2d(x, w, b, y, N, H, W, C, K, F, S_, P, groups, relu != 0);
    return 0;
  });
}

int anx_cpu_maxpool(const float* x, float* y, int N, int H, int W, int C, int F, int S_) {
  return guarded("anx_cpu_maxpool", [&] {
    anx::cpu::maxpool(x, y, N, H, W, C, F, S_);
    return 0;
  });
}

int anx_cpu_lrn(const float* x, float* y, int N, int H, int W, int C, int size, float alpha, float beta, float k,
                int mode) {
  return guarded("anx_cpu_lrn", [&] {
    anx::cpu::lrn(x, y, N, H, W, C, size, alpha, beta, k, static_cast<anx::LrnMode>(mode));
    return 0;
  });
}

int anx_cpu_blocks_forward(const anx_block_c* b1, const anx_block_c* b2, int H, int W, const float* w1,
                           const float* bias1, const float* w2, const float* bias2, const float* x, int N, float* y) {
  return guarded("anx_cpu_blocks_forward", [&] {
    const anx::BlockSpec s1 = from_c(*b1), s2 = from_c(*b2);
    anx::HostWeights hw;
    anx::init_const(hw, s1, s2);
    std::memcpy(hw.w1.data(), w1, hw.w1.size() * sizeof(float));
    std::memcpy(hw.b1.data(), bias1, hw.b1.size() * sizeof(float));
    std::memcpy(hw.w2.data(), w2, hw.w2.size() * sizeof(float));
    std::memcpy(hw.b2.data(), bias2, hw.b2.size() * sizeof(float));
    anx::CpuBlocks eng(s1, s2, H, W, hw);
    eng.forward(x, N, y);
    return 0;
  });
}

int anx_rng_uniform(uint64_t seed, uint64_t stream, float* out, size_t n) {
  for (size_t i = 0; i < n; ++i) out[i] = anx::rng::uniform(seed, stream, i);
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------- cost model
namespace {
int put_json(const std::string& j, char* buf, size_t cap) {
  if (!buf || cap == 0) return fail("anx_cost: no output buffer");
  if (j.size() + 1 > cap) return fail("anx_cost: output buffer too small (" + std::to_string(j.size() + 1) + " bytes)");
  std::memcpy(buf, j.c_str(), j.size() + 1);
  return 0;
}
anx::Workload wl_of(int w) {
  if (w < 0 || w > 2) throw std::invalid_argument("workload must be 0 (dp), 1 (v4) or 2 (v5)");
  return static_cast<anx::Workload>(w);
}
}  // namespace

extern "C" int anx_cost_curve(int workload, const int* nps, int n_nps, int batch, int row_ways, int input_source,
                              int mode, const char* overrides, char* buf, size_t cap) {
  return guarded("anx_cost_curve", [&] {
    std::vector<int> v(nps, nps + std::max(0, n_nps));
    return put_json(anx::model_curve_json(wl_of(workload), v, batch, row_ways,
                                          static_cast<anx::InputSource>(input_source != 0), static_cast<anx::Decomp>(mode),
                                          anx::cost_params(overrides ? overrides : "")),
                    buf, cap);
  });
}

extern "C" int anx_cost_step(int workload, int np, int batch, int row_ways, int input_source, int mode,
                             const char* overrides, char* buf, size_t cap) {
  return guarded("anx_cost_step", [&] {
    return put_json(anx::model_step(wl_of(workload), np, batch, row_ways, static_cast<anx::InputSource>(input_source != 0),
                                    static_cast<anx::Decomp>(mode), anx::cost_params(overrides ? overrides : ""))
                        .json(),
                    buf, cap);
  });
}

extern "C" int anx_cost_pick_row_ways(int workload, int np, int batch, int input_source, int mode, const char* overrides,
                                      int* row_ways) {
  return guarded("anx_cost_pick_row_ways", [&] {
    *row_ways = anx::pick_row_ways(wl_of(workload), np, batch, static_cast<anx::InputSource>(input_source != 0),
                                   static_cast<anx::Decomp>(mode), anx::cost_params(overrides ? overrides : ""));
    return 0;
  });
}

extern "C" int anx_cost_dp_root_batch(int np, int batch, const char* overrides, int* root_batch) {
  return guarded("anx_cost_dp_root_batch", [&] {
    *root_batch = anx::dp_root_batch(np, batch, anx::cost_params(overrides ? overrides : ""));
    return 0;
  });
}
