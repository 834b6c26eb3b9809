// anx/cpu_engine.hpp — host implementation of Blocks 1-2 with the same tile/stage contract as
// BlocksEngine (V1 serial and V2 CPU-rank paths). Parity: alexnetForwardPass
// (v1_serial/src/alexnet_serial.cpp:67-186) and alexnetForwardPassMPI
// (v2_mpi_only/2.2_scatter_halo/src/alexnet_mpi.cpp:4-38).
#pragma once
#include <vector>

#include "anx/engine.hpp"
#include "anx/plan.hpp"

namespace anx {

class CpuBlocks {
 public:
  CpuBlocks(const BlockSpec& b1, const BlockSpec& b2, int H, int W, const HostWeights& w);
  const BlocksDims& dims() const { return d_; }
  void forward(const float* x, int N, float* y);
  void tile_forward(const float* x, int N, const TilePlan& t, float* y);
  // stage1 fills pool1 rows t.p1 of the conv2 input window (zero elsewhere); stage2 consumes it.
  void stage1(const float* x, int N, const TilePlan& t);
  void stage2(int N, const TilePlan& t, float* y);
  float* window_row(const TilePlan& t, int n, int r);
  size_t window_row_floats() const { return static_cast<size_t>(wq_) * d_.C1; }

 private:
  BlockSpec b1_, b2_;
  BlocksDims d_;
  HostWeights w_;
  int wq_;
  std::vector<float> c1_, p1_, q_, c2_, p2_;
};

}  // namespace anx
