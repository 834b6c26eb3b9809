// anx/schedule.hpp — the multi-GPU (V5) data movement of one step as ONE transfer schedule, executed
// by interchangeable transports.
//
// The reference's V5 is a plan (README.md:157-166: device pointers into MPI Scatterv / Isend / Irecv /
// Gatherv); its unused per-layer V4 function shows the shape (v4_mpi_cuda/src/alexnet_mpi_cuda.cu:
// 96-136: halo1 D2H -> MPI -> H2D, halo2 on pool1 rows). Here a step of a hybrid batch x rows plan is:
//
//   Scatter  root X[images, tile.in rows]            -> rank's Tile buffer
//   P1Halo   owner's conv2 window rows (pool1 rows)  -> neighbour's conv2 window (same row group)
//   Gather   rank's Y[images, tile.out rows]         -> root's YFull[images, tile.out rows]
//
// Every transfer is one 2-D block: `height` images of `width` contiguous bytes, image pitches on
// both sides. The schedule is computed once from the plan; the RCCL transport (grouped ncclSend/
// ncclRecv + pack/unpack copies), the peer transport (one hipMemcpy2DAsync straight into the
// IPC-mapped destination) and the host transport (D2H -> TCP -> H2D, V4 staging) all execute
// exactly these lists, which is what lets ranks sharing one GPU (peer) validate what RCCL runs.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>
#include <string>
#include <vector>

#include "anx/comm.hpp"
#include "anx/plan.hpp"

namespace anx {

enum class Phase : int { Scatter = 0, P1Halo = 1, Gather = 2 };
enum class BufId : int { X = 0, Tile = 1, Win = 2, Y = 3, YFull = 4, kCount = 5 };
const char* phase_name(Phase p);

struct Region {
  BufId buf;
  size_t off, pitch;  // bytes
};

struct Transfer {
  Phase phase;
  int src, dst;
  Region from, to;
  size_t width, height;  // bytes per image block, images
  size_t bytes() const { return width * height; }
  std::string str() const;  // "scatter 0->1 w=... h=... from=X+off/pitch to=Tile+off/pitch"
};

// Per-rank buffer geometry the schedule refers to (bytes).
struct StepGeometry {
  size_t in_row, out_row, win_row;  // bytes of one input / output / conv2-window row
  int H, Hp2;                       // input and output image rows
};

struct Schedule {
  std::vector<Transfer> phase[3];  // by Phase
  int np = 1;
};

// Rows of each tile window are those of HybridPlan::tile(rank): Tile holds [n][t.in][row],
// Win the engine's conv2 window [n][t.q][win_row], Y [n][t.out][out_row]; X / YFull are the root's
// full batch [B][H][in_row] / [B][Hp2][out_row].
Schedule make_step_schedule(const HybridPlan& p, const StepGeometry& g);

// Executes the transfers of one phase that involve this rank (src or dst; src == dst ones are a
// local 2-D copy on the compute stream). Ordering contract: on entry the transfer sources are
// complete in stream order on `compute`; on return, work enqueued on `compute` afterwards sees the
// received data. No transport synchronises a stream with the host in steady state except the host
// transport (its data must reach host memory before a socket can send it).
class Transport {
 public:
  virtual ~Transport() = default;
  virtual const char* name() const = 0;
  // Resolve this rank's buffers for both step parities (device pointers; nullptr for buffers the
  // rank does not have; a buffer that does not alternate appears twice). Called once, after
  // allocation, before the first phase; collective over the host channel.
  virtual void bind(const Schedule& s, void* const bufs[2][static_cast<int>(BufId::kCount)], hipStream_t compute) = 0;
  // One phase of step k (parity = k & 1) with the full list of that phase's transfers.
  virtual void run_phase(Phase ph, const std::vector<Transfer>& xs, hipStream_t compute, int parity) = 0;
  // End of a step: every buffer this rank received into has been consumed by the work enqueued on
  // `compute` so far (senders may overwrite them in the next step). On return, work enqueued on
  // `compute` afterwards may overwrite this rank's send buffers (its pushes so far are complete).
  virtual void end_step(hipStream_t compute) = 0;
  virtual void close() {}
  // Record-only mode (no HIP / RCCL / socket call): every transfer is appended to log() — the
  // schedule the transport would execute, for tests and --dry-run.
  bool record_only = false;
  const std::vector<std::string>& log() const { return log_; }

 protected:
  void note(const Transfer& x) { log_.push_back(x.str()); }
  std::vector<std::string> log_;
};

std::unique_ptr<Transport> make_rccl_transport(HostComm& c, int device, int rank);
std::unique_ptr<Transport> make_peer_transport(HostComm& c, int device, int rank);

}  // namespace anx
