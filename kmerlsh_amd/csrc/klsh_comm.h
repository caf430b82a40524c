// Inter-rank exchange for the sharded Cluster() loop (one rank = one klsh_ctx = one GPU).
//
// The loop needs four collective shapes per LSH iteration: an allgather of the
// per-rank key-bin histograms, an all-to-all-v of (key, slot) pairs to the rank that owns each
// key range, an allgather-v of merge deltas (rows rewritten by a merge), and small allgathers of
// counters.  At the end of a call the member links are combined with an element-wise min.
//
// Two implementations behind one interface:
//   RcclComm   one process per GPU, RCCL over xGMI (ncclSend/ncclRecv groups, ncclBroadcast,
//              ncclAllGather, ncclAllReduce) — the product path, bench.py --gpus N.
//   LocalComm  W contexts in ONE process, one host thread each (any devices, including W
//              contexts on the same GPU): peer device-to-device copies behind host barriers.
//              Lets the sharded path be tested bit-for-bit on a single GPU (RCCL refuses two
//              ranks on one device).
// All buffers are device pointers; every call is ordered on the caller's stream.  Sizes are in
// bytes and must agree across ranks as each collective's contract says.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace klsh {

struct Comm {
  int rank = 0;
  int world = 1;
  virtual ~Comm() {}
  virtual const char* kind() const = 0;
  // recv[r * bytes .. (r + 1) * bytes) = rank r's send[0 .. bytes).
  virtual int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // recv[offs[r] .. offs[r] + counts[r]) = rank r's send[0 .. counts[r]); counts/offs identical
  // on every rank.
  virtual int allgatherv(const void* send, void* recv, const size_t* counts, const size_t* offs,
                         hipStream_t s) = 0;
  // To rank r: send[soff[r] .. + scnt[r]); from rank r: recv[roff[r] .. + rcnt[r]).
  virtual int alltoallv(const void* send, const size_t* scnt, const size_t* soff, void* recv,
                        const size_t* rcnt, const size_t* roff, hipStream_t s) = 0;
  // buf[i] = min over ranks of buf[i] (n uint32 elements), in place.
  virtual int allreduce_min_u32(uint32_t* buf, size_t n, hipStream_t s) = 0;
  // After a local failure mid-call: make the group's pending and later collectives fail instead
  // of waiting forever for this rank (RCCL: ncclCommAbort; in-process group: wake every waiter).
  // The communicator is unusable afterwards.
  virtual void abort() = 0;
  // Wait for stream s, which may hold this group's collectives.  RCCL: polls the stream together
  // with ncclCommGetAsyncError, and after an asynchronous error — or no progress for
  // timeout_s seconds (a peer that failed and will never post its half) — aborts the
  // communicator and returns -1, so a rank never blocks forever in a collective its peers
  // abandoned.  The in-process group: a plain stream sync (its collectives are host barriers that
  // an abort already wakes).
  virtual int wait(hipStream_t s) {
    if (hipStreamSynchronize(s) != hipSuccess) {
      err = "stream sync";
      return -1;
    }
    return 0;
  }
  // Wait for event e, recorded on a stream that may hold this group's collectives (as wait()).
  virtual int wait_event(hipEvent_t e) {
    if (hipEventSynchronize(e) != hipSuccess) {
      err = "event sync";
      return -1;
    }
    return 0;
  }
  // Wait until *flag (mapped host memory a kernel on stream s releases) reaches `want`; a stream
  // error — or, RCCL, an asynchronous error or the timeout (as wait()) — ends it with -1.
  virtual int wait_flag(const volatile uint32_t* flag, uint32_t want, hipStream_t s) {
    for (uint64_t spins = 1; (int32_t)(*flag - want) < 0; ++spins) {
      __builtin_ia32_pause();
      if ((spins & 0xFFFu) == 0) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess && (int32_t)(*flag - want) < 0) {
          err = "flag not released by a finished stream";
          return -1;
        }
        if (q != hipSuccess && q != hipErrorNotReady) {
          err = std::string("stream: ") + hipGetErrorString(q);
          return -1;
        }
      }
    }
    return 0;
  }
  double timeout_s = 600.0;  // option "comm_timeout_s"
  bool aborted = false;
  std::string err;
};

// RCCL communicator on the calling thread's current device (one rank per process).
Comm* make_rccl_comm(int rank, int world, const void* unique_id, int device, std::string* err);
int rccl_unique_id(void* out128, std::string* err);

// One in-process group of `world` ranks; returns the rank objects (owned by the caller).
// Each rank's calls must come from its own host thread (they block on each other).
void make_local_comms(int world, Comm** out);

}  // namespace klsh
