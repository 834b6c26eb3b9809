// Per-engine kernel knobs (see anx/knobs.hpp).
#include "anx/knobs.hpp"

#include <cstdlib>
#include <cstring>

#include "anx/bf16_ops.hpp"
#include "anx/ops.hpp"

namespace anx {

namespace {

struct Field {
  const char* name;
  int Knobs::*ip;        // int knobs
  ConvAlgo Knobs::*ap;   // algorithm knobs
  int lo, hi;            // valid range (inclusive)
  const char* env;
};

const Field kFields[] = {
    {"conv1_algo", nullptr, &Knobs::conv1_algo, 0, 2, "ANX_CONV1_ALGO"},
    {"conv2_algo", nullptr, &Knobs::conv2_algo, 0, 2, "ANX_CONV2_ALGO"},
    {"chunk1", &Knobs::chunk1, nullptr, 0, 1 << 30, "ANX_CHUNK1"},
    {"chunk2", &Knobs::chunk2, nullptr, 0, 1 << 30, "ANX_CHUNK2"},
    {"force_vec4", &Knobs::force_vec4, nullptr, -1, 255, nullptr},
    {"force_scalar", &Knobs::force_scalar, nullptr, -1, 255, nullptr},
    {"bf16_glds", &Knobs::bf16_glds, nullptr, 0, 3, "ANX_BF16_GLDS"},
    {"bf16_big", &Knobs::bf16_big, nullptr, -2, 16, "ANX_BF16_BIG"},
    {"bf16_lrn_tile", &Knobs::bf16_lrn_tile, nullptr, 0, 1, nullptr},
    {"bf16_fc_cfg", &Knobs::bf16_fc_cfg, nullptr, -1, 11, "ANX_BF16_FC_CFG"},
    {"bf16_fc_minkt", &Knobs::bf16_fc_minkt, nullptr, 1, 64, nullptr},
    {"bf16_conv1", &Knobs::bf16_conv1, nullptr, 0, 2, "ANX_BF16_CONV1"},
    {"bf16_pool1", &Knobs::bf16_pool1, nullptr, 0, 1, "ANX_BF16_POOL1"},
    {"conv1_occ", &Knobs::conv1_occ, nullptr, 0, 8, "ANX_CONV1_OCC"},
    {"conv2_occ", &Knobs::conv2_occ, nullptr, -1, 8, "ANX_CONV2_OCC"},
    {"conv1_band", &Knobs::conv1_band, nullptr, 0, 2, "ANX_CONV1_BAND"},
    {"fuse_pool1", &Knobs::fuse_pool1, nullptr, 0, 1, "ANX_FUSE_POOL1"},
    {"conv1_fused", &Knobs::conv1_fused, nullptr, 0, 3, "ANX_CONV1_FUSED"},
    {"conv1_pool", &Knobs::conv1_pool, nullptr, 0, 1, "ANX_CONV1_POOL"},
    {"conv1_sub", &Knobs::conv1_sub, nullptr, 0, 1 << 30, "ANX_CONV1_SUB"},
    {"conv2_sub", &Knobs::conv2_sub, nullptr, 0, 1 << 30, "ANX_CONV2_SUB"},
    {"conv2_pool", &Knobs::conv2_pool, nullptr, 0, 1, "ANX_CONV2_POOL"},
    {"conv2_tile", &Knobs::conv2_tile, nullptr, 3, 4, "ANX_CONV2_TILE"},
    {"conv2_sched", &Knobs::conv2_sched, nullptr, 0, 1, "ANX_CONV2_SCHED"},
    {"conv2_in_pg", &Knobs::conv2_in_pg, nullptr, 16, 32, "ANX_CONV2_IN_PG"},
    {"lrn_wgs", &Knobs::lrn_wgs, nullptr, 0, 1 << 20, "ANX_LRN_WGS"},
};

const Field* find(const char* name) {
  if (!name) return nullptr;
  for (const Field& f : kFields)
    if (std::strcmp(f.name, name) == 0) return &f;
  return nullptr;
}

bool valid(const Field& f, int v) {
  if (v < f.lo || v > f.hi) return false;
  if (std::strcmp(f.name, "bf16_glds") == 0) return v == 0 || v == 2 || v == 3;
  if (std::strcmp(f.name, "conv2_in_pg") == 0) return v == 16 || v == 32;
  if (std::strcmp(f.name, "bf16_big") == 0) return v < hip::kConvBf16BigCfgs;
  if (std::strcmp(f.name, "force_vec4") == 0) return hip::conv_variant_valid(0, v);
  if (std::strcmp(f.name, "force_scalar") == 0) return hip::conv_variant_valid(1, v);
  return true;
}

}  // namespace

int set_knob(Knobs& k, const char* name, int value) {
  const Field* f = find(name);
  if (!f || !valid(*f, value)) return -1;
  if (f->ip)
    k.*(f->ip) = value;
  else
    k.*(f->ap) = static_cast<ConvAlgo>(value);
  return 0;
}

int get_knob(const Knobs& k, const char* name, int* value) {
  const Field* f = find(name);
  if (!f || !value) return -1;
  *value = f->ip ? k.*(f->ip) : static_cast<int>(k.*(f->ap));
  return 0;
}

Knobs default_knobs() {
  Knobs k;
  for (const Field& f : kFields) {
    if (!f.env) continue;
    const char* e = std::getenv(f.env);
    if (e && *e) (void)set_knob(k, f.name, std::atoi(e));  // invalid values keep the default
  }
  return k;
}

// Auto: Winograd once a launch covers more than kAutoDirectImages full-height images' worth of
// output rows. Below that the Winograd GEMM grids (64 tiles per workgroup) leave most of the 256
// CUs idle and the direct implicit GEMM wins: 0.081 vs 0.163 ms at batch 1, 0.142 vs 0.169 ms at
// 8, 0.187 (Winograd) vs 0.217 ms at 16 (profiles/r01_algo_crossover.jsonl).
constexpr int kAutoDirectImages = 8;
bool use_winograd(ConvAlgo a, int n, int rows, int full_rows) {
  if (a == ConvAlgo::Direct) return false;
  if (a != ConvAlgo::Auto) return true;
  return static_cast<long>(n) * rows > static_cast<long>(kAutoDirectImages) * full_rows;
}

namespace hip {
size_t occupancy_lds(size_t natural, int wgs) {
  if (wgs <= 0) return natural;
  const size_t cap = 160 * 1024 / static_cast<size_t>(wgs + 1) + 1024;
  return natural > cap ? natural : cap;
}
}  // namespace hip

}  // namespace anx
