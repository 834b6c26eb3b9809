// anx/shapes.hpp — shape algebra and layer specifications shared by host and device code.
//
// Parity: the reference's dim helpers (`calculate_conv_output_dims`
// v1_serial/src/alexnet_serial.cpp:19-36, `convOutDim/poolOutDim` v4_mpi_cuda/include/alexnet.hpp:28-33)
// and its `LayerParams` bag (v1_serial/include/alexnet.hpp:9-24). Unlike the reference, every
// spec is a plain constexpr value type so the planner, kernels and CLI share one table.
#pragma once
#include <cstddef>
#include <cstdint>

namespace anx {

// Guarded like the reference's V4 helpers: a window that does not fit yields 0.
constexpr int conv_out_dim(int d, int f, int s, int p) {
  return (s <= 0 || d + 2 * p < f) ? 0 : (d + 2 * p - f) / s + 1;
}
constexpr int pool_out_dim(int d, int f, int s) {
  return (s <= 0 || d < f) ? 0 : (d - f) / s + 1;
}

// The reference ships two LRN formulas:
//   DivN: x / (k + alpha/N * sum)^beta   (v1_serial/src/layers_serial.cpp:152,167)
//   Raw : x / (k + alpha   * sum)^beta   (v3_cuda_only/src/layers_cuda.cu:138)
enum class LrnMode : int { DivN = 0, Raw = 1 };

struct ConvSpec {
  int C, K, F, S, P, groups;
};
struct PoolSpec {
  int F, S;
};
struct LrnSpec {
  int N;
  float alpha, beta, k;
  LrnMode mode;
};

// One AlexNet "block" as the reference defines it: conv -> ReLU -> maxpool [-> LRN].
struct BlockSpec {
  ConvSpec conv;
  PoolSpec pool;
  bool has_lrn;
  LrnSpec lrn;
};

// Reference hyper-parameters (v1_serial/src/main.cpp:18-43, v4_mpi_cuda/src/main_mpi_cuda.cpp:146-150).
constexpr int kInH = 227, kInW = 227, kInC = 3;
constexpr BlockSpec kBlock1{{3, 96, 11, 4, 0, 1}, {3, 2}, false, {5, 1e-4f, 0.75f, 2.0f, LrnMode::DivN}};
constexpr BlockSpec kBlock2{{96, 256, 5, 1, 2, 1}, {3, 2}, true, {5, 1e-4f, 0.75f, 2.0f, LrnMode::DivN}};

// Per-layer dims of Blocks 1-2 for an H x W input.
struct BlocksDims {
  int H, W;          // input
  int H1, W1;        // conv1 out (55x55)
  int Hp1, Wp1;      // pool1 out (27x27)
  int H2, W2;        // conv2 out (27x27)
  int Hp2, Wp2;      // pool2 / LRN out (13x13)
  int C0, C1, C2;    // channels 3 / 96 / 256
};

constexpr BlocksDims blocks_dims(int H, int W, const BlockSpec& b1 = kBlock1, const BlockSpec& b2 = kBlock2) {
  BlocksDims d{};
  d.H = H;
  d.W = W;
  d.C0 = b1.conv.C;
  d.H1 = conv_out_dim(H, b1.conv.F, b1.conv.S, b1.conv.P);
  d.W1 = conv_out_dim(W, b1.conv.F, b1.conv.S, b1.conv.P);
  d.C1 = b1.conv.K;
  d.Hp1 = pool_out_dim(d.H1, b1.pool.F, b1.pool.S);
  d.Wp1 = pool_out_dim(d.W1, b1.pool.F, b1.pool.S);
  d.H2 = conv_out_dim(d.Hp1, b2.conv.F, b2.conv.S, b2.conv.P);
  d.W2 = conv_out_dim(d.Wp1, b2.conv.F, b2.conv.S, b2.conv.P);
  d.C2 = b2.conv.K;
  d.Hp2 = pool_out_dim(d.H2, b2.pool.F, b2.pool.S);
  d.Wp2 = pool_out_dim(d.W2, b2.pool.F, b2.pool.S);
  return d;
}

static_assert(blocks_dims(227, 227).H1 == 55, "conv1 55");
static_assert(blocks_dims(227, 227).Hp1 == 27, "pool1 27");
static_assert(blocks_dims(227, 227).H2 == 27, "conv2 27");
static_assert(blocks_dims(227, 227).Hp2 == 13, "pool2 13");

// NHWC index (the reference's idx3D, v1_serial/src/layers_serial.cpp:15-18, plus a batch axis).
constexpr size_t nhwc(int n, int h, int w, int c, int H, int W, int C) {
  return ((static_cast<size_t>(n) * H + h) * W + w) * C + c;
}

}  // namespace anx
