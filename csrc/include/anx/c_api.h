/* anx/c_api.h — flat C ABI of libanx (consumed by the Python package through ctypes and by
 * the anx CLI). Every function returns 0 on success or a nonzero status; anx_last_error()
 * returns the message of the last failure on the calling thread. Device pointers and HIP
 * streams are passed as opaque pointers. */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct anx_block_c {
  int C, K, F, S, P, groups; /* conv */
  int pool_F, pool_S;        /* max pool */
  int has_lrn, lrn_N;        /* LRN */
  float lrn_alpha, lrn_beta, lrn_k;
  int lrn_mode; /* 0 = alpha/N (V1/V2), 1 = alpha (V3/V4) */
} anx_block_c;

/* Tile plan rows, half-open: in, c1, p1, q, c2, out (12 ints). */
typedef struct anx_tile_c {
  int in_lo, in_hi, c1_lo, c1_hi, p1_lo, p1_hi, q_lo, q_hi, c2_lo, c2_hi, out_lo, out_hi;
} anx_tile_c;

typedef struct anx_xfer_c {
  int src, dst, lo, hi;
} anx_xfer_c;

const char* anx_last_error(void);
void anx_set_last_error(const char* msg); /* for the companion libraries (libanx_dist) */
int anx_abi_version(void);
int anx_device_count(void);
void anx_default_blocks(anx_block_c* b1, anx_block_c* b2);

/* ---- planner ---- */
/* Fills up to `cap` tiles / transfers; returns counts through the out pointers. */
/* tiles[np]; owned_in[2*np] and owned_p1[2*np] as (lo,hi) pairs; halo lists up to `cap` each. */
int anx_make_plan(int H, int W, int np, int mode, const anx_block_c* b1, const anx_block_c* b2, anx_tile_c* tiles,
                  int* owned_in, int* owned_p1, anx_xfer_c* in_halos, int* n_in_halos, anx_xfer_c* p1_halos,
                  int* n_p1_halos, int cap);

/* ---- cost model (anx/cost.hpp): modelled, not measured ----
 * workload: 0 dp (batch = images per GPU), 1 v4, 2 v5 (batch = global); input_source: 0 local, 1 root;
 * mode: 0 overlap, 1 per_layer; row_ways: -1 = the model's pick; overrides: "name=value;..." over the
 * default CostParams (rate=IMG:IPS,... for the rate table). anx_cost_curve writes the JSON curve over
 * nps[0..n_nps) into buf; anx_cost_step one step's JSON; anx_cost_pick_row_ways the chosen split. */
int anx_cost_curve(int workload, const int* nps, int n_nps, int batch, int row_ways, int input_source, int mode,
                   const char* overrides, char* buf, size_t cap);
int anx_cost_step(int workload, int np, int batch, int row_ways, int input_source, int mode, const char* overrides,
                  char* buf, size_t cap);
int anx_cost_pick_row_ways(int workload, int np, int batch, int input_source, int mode, const char* overrides,
                           int* row_ways);
/* dp: images rank 0 computes per step when every peer has `batch` (its ingest slowdown shed). */
int anx_cost_dp_root_batch(int np, int batch, const char* overrides, int* root_batch);

/* ---- engine (Blocks 1-2) ---- */
/* Hybrid batch x rows plan (anx/plan.hpp make_hybrid_plan). Per rank r (arrays of np):
   group[r], index[r] (position in its group), img[2r..2r+1] (its image range), tile[r] (its rows);
   per group g (arrays of np, first `*groups` used): gsize[g]. redundancy: conv1 rows computed over
   one device's, minus 1. */
int anx_make_hybrid_plan(int H, int W, int np, int batch, int row_ways, int mode, const anx_block_c* b1,
                         const anx_block_c* b2, int* groups, int* group, int* index, int* img, int* gsize,
                         anx_tile_c* tile, double* redundancy);
int anx_engine_create(void** out, const anx_block_c* b1, const anx_block_c* b2, int H, int W, const float* w1,
                      const float* bias1, const float* w2, const float* bias2, int max_batch, int impl);
int anx_engine_destroy(void* e);
int anx_engine_forward(void* e, const float* x, int N, float* y, void* stream);
int anx_engine_tile_forward(void* e, const float* x, int N, const anx_tile_c* t, float* y, void* stream);
int anx_engine_stage1(void* e, const float* x, int N, const anx_tile_c* t, void* stream);
int anx_engine_stage2(void* e, int N, const anx_tile_c* t, float* y, void* stream);
/* conv2 input window geometry: pointer of (image n, pool1 row r), row stride and image stride (floats). */
int anx_engine_window(void* e, const anx_tile_c* t, int n, int r, float** ptr, size_t* row_floats,
                      size_t* image_floats);

/* ---- full AlexNet bf16 engine (extension) ----
 * weights: 8 KCFF/[out][in] fp32 host arrays (conv1..5, fc6..8), biases: 8 fp32 host arrays. */
int anx_full_weight_sizes(int classes, int groups2, size_t* wn, size_t* bn);
int anx_full_create(void** out, const float* const* weights, const float* const* biases, int classes,
                    int max_batch, int groups2, int lrn_mode);
int anx_full_destroy(void* e);
int anx_full_forward(void* e, const float* x, int N, float* logits, void* stream);
/* forward that records the engine's mark event half-way (after Conv2 + Pool2/LRN of the first chunk);
   anx_full_wait_mark makes `stream` wait for the last recorded mark of engine e. */
int anx_full_forward_mark(void* e, const float* x, int N, float* logits, void* stream);
int anx_full_wait_mark(void* e, void* stream);

/* ---- host engine (same contract as the device engine; V1 / V2 CPU ranks) ---- */
int anx_cpu_engine_create(void** out, const anx_block_c* b1, const anx_block_c* b2, int H, int W, const float* w1,
                          const float* bias1, const float* w2, const float* bias2);
int anx_cpu_engine_destroy(void* e);
int anx_cpu_engine_tile_forward(void* e, const float* x, int N, const anx_tile_c* t, float* y);
int anx_cpu_engine_stage1(void* e, const float* x, int N, const anx_tile_c* t);
int anx_cpu_engine_stage2(void* e, int N, const anx_tile_c* t, float* y);
int anx_cpu_engine_window(void* e, const anx_tile_c* t, int n, int r, float** ptr, size_t* row_floats,
                          size_t* image_floats);
/* strided host copy (memcpy per row) */
int anx_memcpy2d_host(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes, size_t height);

/* ---- memory ---- */
/* hipMemcpy2DAsync (kind = default: direction inferred from the pointers). */
int anx_memcpy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes, size_t height,
                       void* stream);

/* ---- device ops ---- */
int anx_conv2d_direct(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C, int K,
                      int F, int S, int P, int groups, int relu, void* stream);
int anx_relu(float* x, size_t n, void* stream);
/* copy on exactly `workgroups` workgroups (tools/probe_ingest.py); bytes % 16 == 0, 16-B aligned */
int anx_channel_copy(void* dst, const void* src, size_t bytes, int workgroups, void* stream);
int anx_maxpool_direct(const float* x, float* y, int N, int H, int W, int C, int F, int S, void* stream);
int anx_lrn_direct(const float* x, float* y, int N, int H, int W, int C, int size, float alpha, float beta, float k,
                   int mode, void* stream);
/* out view: base + ((n*Hb + h + h_off)*Wb + w + w_off)*Cb + c_off + c */
int anx_maxpool(const float* x, int N, int H, int W, int C, int F, int S, float* out, int Hb, int Wb, int Cb,
                int h_off, int w_off, int c_off, void* stream);
int anx_maxpool_lrn(const float* x, float* y, int N, int H, int W, int C, int F, int S, int size, float alpha,
                    float beta, float k, int mode, void* stream);
/* MFMA conv: plan -> sizes; pack on host; run. plan_out: 16 ints (opaque, pass back unchanged). */
int anx_conv_plan(int N, int Hp, int Wp, int C, int K, int F, int S, int groups, int* plan_out,
                  size_t* packed_floats, size_t* koff_ints);
int anx_conv_pack(const int* plan, const float* w_kcff, float* packed, int* koff);
/* Per-engine kernel knobs: the field names of anx::Knobs (anx/knobs.hpp). set returns non-zero for an
   unknown name, an out-of-range value or a failed workspace re-allocation (the knob is then unchanged);
   it may free buffers a previously captured HIP graph names: re-capture after it. */
int anx_engine_set_knob(void* engine, const char* name, int value);
int anx_engine_get_knob(void* engine, const char* name, int* value);
/* bf16 activation tap `i` of the last forward (FullEngine::tap) into dst; *elems = per-image count */
int anx_full_tap(void* engine, int i, int N, void* dst, size_t* elems, void* stream);
int anx_full_set_knob(void* engine, const char* name, int value);
int anx_full_get_knob(void* engine, const char* name, int* value);
/* the defaults a new engine starts from (built-in values overridden by ANX_* environment variables) */
int anx_default_knob(const char* name, int* value);
/* Conv1 by polyphase Winograd on device buffers (test entry; allocates and frees its workspaces,
   synchronises `stream`): x [N,Hin,W,3], KCFF weights on the HOST, y [N,H1,W1,K]. */
int anx_conv1_wino(const float* x, int N, int Hin, int W, const float* w_kcff, int K, int F, const float* bias,
                   float* y, int relu, void* stream);
/* Conv2-shaped 5x5/1 conv by Winograd F(3x3,5x5) on device buffers (test entry; allocates, syncs):
   x [N,Hq,Wq,C] (padding already in the window), KCFF weights on the HOST, y [N,Hq-4,Wq-4,K]. */
int anx_conv2_wino(const float* x, int N, int Hq, int Wq, int C, const float* w_kcff, int K, int groups,
                   const float* bias, float* y, int relu, void* stream);
// The same with the Winograd output tile m = 3 (F(3x3,5x5)) or 4 (F(4x4,5x5), one group of 96 channels).
int anx_conv2_wino_tile(const float* x, int N, int Hq, int Wq, int C, const float* w_kcff, int K, int groups,
                        const float* bias, float* y, int relu, void* stream, int m);
int anx_conv2d_mfma(const int* plan, const float* x, const float* wpacked, const int* koff, const float* bias,
                    float* out, int Hb, int Wb, int Cb, int h_off, int w_off, int c_off, int relu, void* stream);

/* ---- V5 device-resident runtime (libanx_dist.so: anx/v5.hpp) ----
 * anx_v5_create is collective over the `world` ranks (TCP bootstrap at master_addr:master_port, then
 * the transport: RCCL or peer IPC). Weights are read on rank 0 only (others may pass NULL).
 * mode: 0 overlap, 1 per_layer; row_ways: -1 the cost model's pick, 0 batch first, r > 0 groups of r
 * ranks; transport: "auto" | "rccl" | "peer" | "loopback"; chunks: 0 auto; pipeline: -1 auto, 0 off,
 * 1 on; peer_sync: "" | "flags" | "notes"; input_source: 0 local (device-resident, placed once by
 * set_input), 1 root (scattered every step); lanes: stream lanes of a halo-free rank (0 = default 2);
 * keep_log: keep the transport's transfer log (anx_v5_log); root_images: a batch split's rank-0 share
 * (the dp headline's root shedding; -1 = even). */
int anx_v5_create(void** out, int rank, int world, int local_rank, int local_world, int nnodes,
                  const char* master_addr, int master_port, double timeout_s, const anx_block_c* b1,
                  const anx_block_c* b2, int H, int W, const float* w1, const float* bias1, const float* w2,
                  const float* bias2, int batch, int row_ways, int mode, const char* transport, int chunks,
                  int pipeline, int poison, int impl, const char* peer_sync, int input_source, int lanes,
                  int keep_log, int root_images);
int anx_v5_log(void* h, char* buf, size_t cap); /* this rank's issued transfers, one per line */
int anx_v5_destroy(void* h);
int anx_v5_set_input(void* h, const float* host_x); /* collective; rank 0's batch, others NULL */
int anx_v5_step(void* h, int steps);                /* enqueue `steps` steps, no host sync */
int anx_v5_sync(void* h);
int anx_v5_output(void* h, float* host_y);          /* rank 0: last step's output */
/* JSON objects into buf (truncated to cap): per-phase mean ms since the last reset / the layout */
int anx_v5_phases(void* h, char* buf, size_t cap, int reset);
int anx_v5_describe(void* h, char* buf, size_t cap);
/* Record-only schedule, no GPU: rank < 0 -> every transfer of one step (scatter with root input,
 * halo chunks, gather), else the transfers rank `rank`'s transport issues, in order; one per line. */
int anx_v5_schedule(int np, const anx_block_c* b1, const anx_block_c* b2, int H, int W, int batch, int row_ways,
                    int mode, int chunks, int rank, const char* transport, int input_source, char* buf, size_t cap);

/* ---- V4 host-staged runtime (libanx_dist.so: anx/v4.hpp) ----
 * Collective create; the batch and the output live in a shared pinned host segment every rank maps
 * (anx_v4_segment): write the input, call anx_v4_input_ready (collective), step, anx_v4_sync_all
 * (collective), read the output. row_ways: -1 the cost model's pick, 0 batch first, r > 0 groups of r ranks. */
int anx_v4_create(void** out, int rank, int world, int local_rank, int local_world, int nnodes,
                  const char* master_addr, int master_port, double timeout_s, const anx_block_c* b1,
                  const anx_block_c* b2, int H, int W, const float* w1, const float* bias1, const float* w2,
                  const float* bias2, int batch, int row_ways, int chunks, int impl);
int anx_v4_destroy(void* h);
int anx_v4_segment(void* h, float** input, const float** output);
int anx_v4_input_ready(void* h);
int anx_v4_step(void* h, int steps);
int anx_v4_sync_all(void* h);
int anx_v4_phases(void* h, char* buf, size_t cap, int reset); /* h2d / compute / d2h ms per step */
int anx_v4_describe(void* h, char* buf, size_t cap);
/* GB/s of one H2D of this rank's whole share (its link alone, no compute): the H2D bound */
int anx_v4_probe_h2d(void* h, int reps, double* gbps);

/* ---- CPU reference ---- */
int anx_cpu_conv2d(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C, int K, int F,
                   int S, int P, int groups, int relu);
int anx_cpu_maxpool(const float* x, float* y, int N, int H, int W, int C, int F, int S);
int anx_cpu_lrn(const float* x, float* y, int N, int H, int W, int C, int size, float alpha, float beta, float k,
                int mode);
/* Full Blocks 1-2 on the host (V1): x [N,H,W,C0] -> y [N,Hp2,Wp2,C2]. */
int anx_cpu_blocks_forward(const anx_block_c* b1, const anx_block_c* b2, int H, int W, const float* w1,
                           const float* bias1, const float* w2, const float* bias2, const float* x, int N, float* y);

/* ---- deterministic init (bit-identical to anx.utils.init) ---- */
int anx_rng_uniform(uint64_t seed, uint64_t stream, float* out, size_t n);

#ifdef __cplusplus
}
#endif
