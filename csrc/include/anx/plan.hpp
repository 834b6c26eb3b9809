// anx/plan.hpp — exact receptive-field decomposition planner for AlexNet Blocks 1-2.
//
// The reference sizes halos heuristically (F/2 rows, zero-filled even where conv1 has P=0) and
// trims by ad-hoc formulas (v2_mpi_only/2.2_scatter_halo/src/main.cpp:119-230,
// v4_mpi_cuda/src/main_mpi_cuda.cpp:65-122), which is why its np>=2 outputs have the wrong
// shape. Its unused alexnetForwardPassMPI_CUDA had the right
// idea — map a rank's rows through each layer (v4_mpi_cuda/src/alexnet_mpi_cuda.cu:27-83).
// This planner does that exactly: partition the OUTPUT rows, back-propagate the receptive
// field through pool2 -> conv2 -> pool1 -> conv1, clip to the valid ranges, and record which
// rows of which layer every rank computes, needs, and must receive from whom.
//
// All ranges are half-open [lo, hi) in the global row index space of the named layer.
#pragma once
#include <vector>

#include "anx/shapes.hpp"

namespace anx {

struct RowRange {
  int lo = 0, hi = 0;
  int size() const { return hi > lo ? hi - lo : 0; }
  bool empty() const { return hi <= lo; }
};

struct TilePlan {
  RowRange in;   // input image rows the tile reads
  RowRange c1;   // conv1 output rows computed
  RowRange p1;   // pool1 rows computed locally from `in`
  RowRange q;    // conv2 input window (pool1 index space; rows outside [0,Hp1) are zero padding)
  RowRange c2;   // conv2 output rows computed
  RowRange out;  // pool2/LRN output rows produced (= owned)
};

// A halo transfer of pool1 rows [rows.lo, rows.hi) from rank `src` to rank `dst`.
struct HaloXfer {
  int src, dst;
  RowRange rows;
};

enum class Decomp : int {
  Overlap = 0,   // each rank gets every input row it needs (redundant halo); no mid-network exchange
  PerLayer = 1,  // ranks own pool1 rows; exchange pool1 halos before conv2 (V5)
};

struct DecompPlan {
  int np = 1;
  Decomp mode = Decomp::Overlap;
  BlocksDims dims{};
  BlockSpec b1 = kBlock1, b2 = kBlock2;
  std::vector<TilePlan> tiles;     // one per rank
  // Scatter + halo-exchange formulation of the input distribution (V2.2 / V4 shape): a
  // disjoint partition of the input rows plus the input rows each rank must then receive.
  std::vector<RowRange> owned_in;
  std::vector<HaloXfer> in_halos;
  // PerLayer (V5): disjoint ownership of pool1 rows and the pool1 rows exchanged before conv2.
  std::vector<RowRange> owned_p1;
  std::vector<HaloXfer> p1_halos;
};

// Split `n` items over `np` ranks: the first n % np ranks get one extra (the reference's
// Scatterv split rule, v2_mpi_only/2.2_scatter_halo/src/main.cpp:102-109).
std::vector<RowRange> split_rows(int n, int np);

// Receptive-field mapping helpers for one conv/pool layer (global row spaces).
RowRange conv_rows_needed(RowRange out, int F, int S, int P, int in_rows);  // input rows for conv outputs (clipped)
RowRange pool_rows_needed(RowRange out, int F, int S, int in_rows);

DecompPlan make_plan(int H, int W, int np, Decomp mode, const BlockSpec& b1 = kBlock1,
                     const BlockSpec& b2 = kBlock2);

// A plan is valid if the tiles' outputs partition [0, Hp2) and every layer window is
// consistent with the layer algebra. Returns an empty string when valid, else a message.
const char* check_plan(const DecompPlan& p);

// Redundant Conv1 work of a row decomposition: sum over ranks of the conv1 rows each computes,
// divided by the image's conv1 rows, minus 1 (0 = no row is computed twice). Overlap tiles
// recompute their neighbours' rows (np = 8: 1.38); per-layer tiles only at the pool1 seams.
double conv1_redundancy(const DecompPlan& p);

// Hybrid batch x rows decomposition. The reference only splits image rows
// (v2_mpi_only/2.2_scatter_halo/src/main.cpp:100-249); images are independent, so the batch is split
// first and rows only where there are fewer images than ranks (or when asked):
//   row_ways == 0 (auto): batch >= np -> np groups of 1 rank, images split over them (pure batch);
//                         batch <  np -> `batch` groups of one image each, the ranks split over the
//                         groups as evenly as possible (sizes differ by at most one), rows inside.
//   row_ways == r > 0   : np / r groups of r ranks (np % r == 0), images split over the groups,
//                         each group row-decomposes its images r ways (r == np: the reference's
//                         pure row split of the whole batch).
// Every rank computes images `images[group_of[rank]]` x tile rows_plan(rank).
struct HybridPlan {
  int np = 1, batch = 1, groups = 1;
  std::vector<RowRange> images;      // per group: its image range (empty when batch < groups)
  std::vector<int> group_first;      // per group: its first rank (ranks of a group are contiguous)
  std::vector<int> group_size;       // per group: its number of ranks
  std::vector<int> group_of, index_in_group;  // per rank
  std::vector<DecompPlan> row_plans;  // per group: the row plan over group_size[g] ranks
  const TilePlan& tile(int rank) const { return row_plans[group_of[rank]].tiles[index_in_group[rank]]; }
};
// Returns false (plan untouched) for an invalid request (np < 1, batch < 1, row_ways > np or not
// dividing np).
bool make_hybrid_plan(int H, int W, int np, int batch, int row_ways, Decomp mode, HybridPlan& out,
                      const BlockSpec& b1 = kBlock1, const BlockSpec& b2 = kBlock2);
// Conv1 rows computed by all ranks over the batch, relative to one device computing it: 0 for a
// pure batch split.
double conv1_redundancy(const HybridPlan& p);

}  // namespace anx
