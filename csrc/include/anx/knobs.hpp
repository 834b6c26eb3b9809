// anx/knobs.hpp — per-engine kernel selection and tuning.
//
// Every algorithm choice and A/B knob of the compute path lives in one value type that an engine
// owns (BlocksEngine, FullEngine) and passes to the launchers it calls. Two engines in one process
// can therefore run different kernels (stream lanes, A/B arms, tests), and nothing a launch reads
// is process-wide mutable state. Environment variables (ANX_*) only seed default_knobs(), once per
// engine construction.
//
// The reference has no run-time configuration at all: every dim and parameter is hard-coded in each
// version's main() (v1_serial/src/main.cpp:18-43, v4_mpi_cuda/src/main_mpi_cuda.cpp:146-150).
#pragma once

namespace anx {

// Algorithm for a convolution on the Mfma path. Auto = Winograd when eligible and the launch is
// larger than 8 images' worth of output rows (use_winograd), the direct implicit GEMM below that.
enum class ConvAlgo : int { Auto = 0, Direct = 1, Winograd = 2 };

// Three kinds of field (round 5: the measured-worse variants are gone from libanx; the split-bf16
// GEMMs, the U-in-registers Conv1 and the activation-streaming FC kernel were deleted):
//   production  the defaults every bench and driver run launches, and their shape fallbacks;
//   oracle      a simpler kernel kept as the bitwise / tolerance reference of a fast one in the GPU tests:
//               conv*_algo = direct, conv1_band = 0 (per-tile gathers), bf16_glds = 0 with bf16_big = -2
//               (the register-staged 128x128 bf16 kernel), fuse_pool1 / conv1_pool / conv2_pool / conv1_fused = 0;
//   tuning      launch geometry (chunks, sub-chunks, occupancy caps, forced tile configs) for A/B runs.
struct Knobs {
  ConvAlgo conv1_algo = ConvAlgo::Auto;  // Conv1: polyphase Winograd F(3x3,3x3) / direct implicit GEMM
  ConvAlgo conv2_algo = ConvAlgo::Auto;  // Conv2: Winograd F(3x3,5x5) / direct implicit GEMM
  int chunk1 = 0;          // images per stage-1 launch (0 = whole batch up to the 32-bit index chunk)
  int chunk2 = 0;          // images per stage-2 launch
  int force_vec4 = -1;     // conv_mfma tile variant override for Cg % 4 == 0 convs (-1 = heuristic)
  int force_scalar = -1;   // conv_mfma tile variant override for scalar-gather convs
  int bf16_glds = 2;       // bf16 128x128 kernel: 2 / 3 LDS-DMA ring slots; 0 register-staged (oracle)
  int bf16_big = -1;       // bf16 conv layers on the wide-tile kernel (conv_bf16_big.hip): -1 cost model
                           // picks the config, 0.. force that config; -2 off (the 128x128 kernels: oracle)
  int bf16_fc_cfg = -1;    // bf16 FC layers: force this wide-tile config (A/B; -1 = cfg 8, 256x64 3-stage)
  int bf16_fc_minkt = 4;   // bf16 FC layers: K tiles per split-K slice at least this many (fewer slices, less
                           // reduce; 8 / 16 measured no better: profiles/r04_bf16_fc_minkt_ab.jsonl)
  int bf16_lrn_tile = 0;   // bf16 pool2+LRN: 1 = the generic LDS-tile kernel instead of the C=256 wave kernel
  int bf16_conv1 = 2;      // bf16 Conv1 (polyphase): 2 = the persistent row-band kernel on the fp32 image
                           // (conv1_bf16_ring.hip: space-to-depth + bf16 inside, rows in an LDS ring, weights
                           // resident; 362 k vs 343 k images/s, profiles/r04_bf16_ring_v2_bench_ab.jsonl),
                           // 1 = the same on the s2d4 polyphase copy, 0 = s2d4 + the implicit-GEMM tile kernels
  int bf16_pool1 = 1;      // bf16 pool1: 1 = in the Conv1 ring kernel's epilogue (bf16_conv1 2, one workgroup per
                           // image: the 55x55 map never reaches HBM), 0 = Conv1 writes it and maxpool_bf16 reads it
  int conv1_occ = 0;       // cap on the Conv1 Winograd GEMM's workgroups per CU (LDS padding; 0 = none: 4)
  int conv2_occ = -1;      // ... and Conv2's (0 = none: 2; -1 = auto: 1 when the launch has <= one workgroup per
                           // CU); a cap leaves room for a concurrent lane's kernels
  int conv1_band = 2;      // Conv1 polyphase input transform, band kernel (a tile row's image rows staged in LDS):
                           // 2 = all 4 phase rows x half the tile columns (each 192-B V segment written whole),
                           // 1 = 2 phase rows x all columns, 0 = per-tile gathers from global memory
  int fuse_pool1 = 1;      // tile_forward of a tile that computes every pool1 row its conv2 window needs: pool1
                           // fused into the Winograd input transform (no window round trip), 0 = pool1 kernel
  int conv1_fused = 2;     // Conv1 as one kernel (conv1_fused.hip: V built in LDS inside the GEMM, 32 tiles x 96
                           // filters per workgroup; bench step 277-278 k vs 252-254 k images/s,
                           // profiles/r04_conv1_fused_v3_bench_ab.jsonl), 0 = the band transform kernel + GEMM (the
                           // general path: also every conv1 with K != 96). 2 (default since round 6) = with pool1 in
                           // the epilogue, a private U ring per wave (each wave DMAs its own filter rows and waits
                           // with its own vmcnt: barriers only where V is published, 5 instead of 25; main loop
                           // 48.1 k -> 44.2 k clk per workgroup, bench 335-339 k vs 325-330 k images/s,
                           // profiles/r06_conv1_upw/); 1 = the shared 3-slot ring (every wave's DMA, one barrier
                           // per point)
  int conv1_pool = 1;      // fused tile_forward of whole images: pool1 in the one-kernel Conv1's epilogue (conv1_fused 1;
                           // the 55x55 map stays in LDS, pooled pixels go to the conv2 window, straddling windows'
                           // partial maxima to a side buffer merged by the Conv2 input transform), 0 = Conv1 writes its
                           // map and the input transform pools it
  int conv1_sub = 0;       // fused tile_forward: images per Conv1 (input transform + GEMM) launch pair inside a
                           // chunk (0 = the whole chunk); the V workspace is rewritten in place per sub-chunk, so
                           // a small one is written and re-read inside the 256 MB Infinity Cache
  int conv2_sub = 0;       // ... and per (pool1 + Conv2 input transform, Conv2 GEMM) pair
  int conv2_pool = 1;      // 1 (default since round 6) = for whole images on F(4x4,5x5) with LRN over 256 channels, pool2
                           // in the Conv2 GEMM's epilogue (the 27x27 map never reaches HBM: -125 MB per 128 images;
                           // straddling windows' partial maxima to a side buffer merged by the LRN kernel). Round 5
                           // measured it level with the compiler-scheduled GEMM (320.8-322.1 k vs 322.1-323.0 k,
                           // profiles/r05_conv2_pool/); with the hand-scheduled K slice it is +3 % (349.0-350.4 k vs
                           // 338.1-340.9 k, profiles/r06_conv2_pool/). 0 = the GEMM writes its map and maxpool_lrn pools it
  int conv2_tile = 4;      // Conv2 Winograd output tile: 4 = F(4x4,5x5) (64 points per 16 outputs: 21 % fewer
                           // multiplies, 16x16x4 MFMAs, wino_gemm16.hpp; one group of 96 channels only, else 3;
                           // bench step 305-309 k vs 293 k images/s, profiles/r05_f45/), 3 = F(3x3,5x5) (49
                           // points, 32x32x2 MFMAs: grouped Conv2 and the A/B arm)
  int conv2_in_pg = 32;    // tuning: channels per workgroup of the Conv2 input transform after the pooled Conv1 (32: 31 KiB of
                           // LDS; 16: 15.5 KiB, fits on a CU beside a per-wave-ring Conv1 workgroup)
  int conv2_sched = 1;     // F(4x4,5x5) GEMM K-slice schedule: 1 = hand-scheduled (wino_gemm16_sched.inc: fragment
                           // reads two groups ahead with counted lgkmcnt, alternating accumulators, the fold as one
                           // packed burst at the slice start; bitwise identical), 0 = the compiler's schedule
  int lrn_wgs = 256;       // grid cap of the pool2-merge + LRN kernel after the pooled Conv2 GEMM (0 = one wave per pixel
                           // pair, 1352 workgroups per 64 images): under the bench's co-running lanes fewer, longer
                           // workgroups wait less for CU slots (+0.8-1.5 %, profiles/r06_lrn_grid/); same bits
};

// Built-in defaults, overridden by ANX_CONV1_ALGO, ANX_CONV2_ALGO, ANX_CHUNK1, ANX_CHUNK2,
// ANX_BF16_GLDS, ANX_BF16_BIG, ANX_CONV1_OCC, ANX_CONV2_OCC, ANX_CONV1_BAND, ANX_FUSE_POOL1,
// ANX_CONV1_SUB, ANX_CONV2_SUB, ANX_CONV1_FUSED, ANX_CONV1_POOL, ANX_CONV2_POOL, ANX_CONV2_TILE,
// ANX_CONV2_SCHED, ANX_LRN_WGS when set.
Knobs default_knobs();

// Name-based access for the C ABI / Python (names: the field names above). Returns 0, or -1 for
// an unknown name or an out-of-range value (the knob is then unchanged).
int set_knob(Knobs& k, const char* name, int value);
int get_knob(const Knobs& k, const char* name, int* value);

// Whether a launch of n images x `rows` output rows of a conv whose full image has `full_rows`
// rows runs Winograd under algorithm a (Auto: above 8 full images' worth of rows).
bool use_winograd(ConvAlgo a, int n, int rows, int full_rows);

}  // namespace anx
