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
// ncclRecv + pack/unpack copies) and the peer transport (one hipMemcpy2DAsync straight into the
// IPC-mapped destination, device-side flags for ordering) execute exactly these lists, which is what
// lets ranks sharing one GPU (peer) validate what RCCL runs.
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
  // Pipelined halos (anx/v5.hpp): a phase list is cut into chunks of images; `chunk` is the chunk
  // index (-1: whole phase), `seq` the index of the uncut transfer in its phase list and `img0` the
  // first image of this block inside it.
  int chunk = -1, seq = -1;
  size_t img0 = 0;
  size_t bytes() const { return width * height; }
  // "scatter 0->1 w=... h=... from=X+off/pitch to=Tile+off/pitch" ("halo_p1#c ..." for chunk c)
  std::string str() const;
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

// Chunk c of `chunks` of a phase list: every transfer restricted to images
// [height * c / chunks, height * (c + 1) / chunks) of its block (empty blocks dropped). Each group's
// images are cut the same way by the compute stream (v5.cpp), so chunk c of a halo carries exactly
// the rows stage1 produced for chunk c.
std::vector<Transfer> chunk_of(const std::vector<Transfer>& xs, int c, int chunks);

// Executes the transfers of one phase that involve this rank (src or dst; src == dst ones are a
// local 2-D copy on the given stream). Ordering contract: on entry the transfer sources are
// complete in stream order on the given stream; on return, work enqueued on that stream afterwards
// sees the received data AND this rank's sends of the phase are complete (so it may overwrite their
// sources). No transport synchronises a stream with the host in steady state.
class Transport {
 public:
  virtual ~Transport() = default;
  virtual const char* name() const = 0;
  // how receives are ordered after sends: "events" (RCCL stream), "flags" / "notes" (peer)
  virtual const char* ordering() const = 0;
  // Resolve this rank's buffers for both step parities (device pointers; nullptr for buffers the
  // rank does not have; a buffer that does not alternate appears twice). Called once, after
  // allocation, before the first phase; collective over the host channel.
  virtual void bind(const Schedule& s, void* const bufs[2][static_cast<int>(BufId::kCount)], hipStream_t compute) = 0;
  // Device-to-device broadcast of `bytes` at `buf` from rank `root` (collective; synchronous: on
  // return every rank's buffer holds the root's bytes). Weights reach the ranks this way.
  virtual void bcast(void* buf, size_t bytes, int root) = 0;
  // One phase of step k (parity = k & 1) with the full list of that phase's transfers (or one chunk
  // of it, see chunk_of: every rank must issue the same sequence of phase / chunk calls).
  virtual void run_phase(Phase ph, const std::vector<Transfer>& xs, hipStream_t compute, int parity) = 0;
  // Collective teardown (unmap peers' buffers, free own ones).
  virtual void close() {}
  // Fail-stop (not collective): release every device-side wait of this rank's streams on its peers so
  // they drain (RCCL: ncclCommAbort; device flags: every flag word this rank waits on, and the ones its
  // peers wait on, raised to the maximum). The transport is unusable afterwards; close() skips the
  // collective part.
  virtual void abort() {}
  // Record-only mode (no HIP / RCCL / socket call): every transfer is appended to log() — the
  // schedule the transport would execute, for tests and --dry-run.
  bool record_only = false;
  // Keep the log in live mode too (tests: the transfers a live run issued == the record-only schedule).
  bool keep_log = false;
  const std::vector<std::string>& log() const { return log_; }
  // transfers this rank took part in so far (every mode)
  size_t issued() const { return issued_; }

 protected:
  void note(const Transfer& x) {
    ++issued_;
    if (record_only || keep_log) log_.push_back(x.str());
  }
  std::vector<std::string> log_;
  size_t issued_ = 0;
};

// `c` may be null for a record-only transport (no collective is issued then). loopback: over the
// loopback DeviceComm (ranks sharing one GPU) instead of an RCCL communicator; name "rccl-loopback".
std::unique_ptr<Transport> make_rccl_transport(HostComm* c, int device, int rank, bool loopback = false);
// Host buffers on CPU ranks: the same transfer lists moved by HostComm's grouped point-to-point (TCP;
// strided blocks packed / unpacked through staging), local blocks by memcpy. Blocking: run_phase
// returns with the phase complete. Name "host". The V5 runtime's CPU mode (V5Options::host) runs on
// it, which is how the CPU multi-rank tests rehearse the schedule the GPU transports execute.
std::unique_ptr<Transport> make_host_transport(HostComm* c, int rank);
// Peer ordering: "flags" (default where the device supports hipStreamWaitValue32) = the sender's
// stream writes a sequence number into the receiver's IPC-mapped flag word after its pushes and the
// receiver's stream waits for it on the device (no host involvement per phase); "notes" = IPC
// events + a 4-byte host note per phase over the TCP channel. "" = ANX_PEER_SYNC or the default.
std::unique_ptr<Transport> make_peer_transport(HostComm* c, int device, int rank, const std::string& sync = "");

}  // namespace anx
