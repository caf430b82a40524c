// Inter-rank exchange for the sharded loop: RCCL (product) and in-process (tests).  See
// klsh_comm.h.
#include "klsh_comm.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "klsh_internal.h"

namespace klsh {

// ============================================================================== RCCL ===========
namespace {

struct RcclComm final : Comm {
  ncclComm_t nc = nullptr;
  const char* kind() const override { return "rccl"; }
  ~RcclComm() override {
    if (nc) (void)ncclCommDestroy(nc);
  }
  void abort() override {
    aborted = true;
    if (nc) (void)ncclCommAbort(nc);
    nc = nullptr;
  }
  int wait(hipStream_t s) override {
    return poll([&] { return hipStreamQuery(s); });
  }
  int wait_event(hipEvent_t e) override {
    return poll([&] { return hipEventQuery(e); });
  }
  int wait_flag(const volatile uint32_t* flag, uint32_t want, hipStream_t s) override {
    // the flag first; the stream (errors) and the communicator every 256 polls, as wait()
    uint32_t spins = 0;
    return poll([&] {
      if ((int32_t)(*flag - want) >= 0) return hipSuccess;
      if ((++spins & 63u) != 0) return hipErrorNotReady;  // (the stream only now and then)
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) return (int32_t)(*flag - want) >= 0 ? hipSuccess : hipErrorUnknown;
      return q;
    });
  }
  template <class Query>
  int poll(Query query) {
    if (aborted) return check(ncclSuccess, "wait");
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t polls = 0;; ++polls) {
      const hipError_t q = query();
      if (q == hipSuccess) return 0;
      if (q != hipErrorNotReady) {
        err = std::string("stream: ") + hipGetErrorString(q);
        abort();
        return -1;
      }
      if ((polls & 255u) == 0) {
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(nc, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress)) {
          err = std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae);
          abort();
          return -1;
        }
        const double secs =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (secs > timeout_s) {
          err = "collective timed out after " + std::to_string((int)secs) +
                " s (a peer rank failed or stopped); communicator aborted";
          abort();
          return -1;
        }
      }
      __builtin_ia32_pause();
    }
  }
  int check(ncclResult_t r, const char* what) {
    if (aborted) {
      err = std::string(what) + ": communicator aborted";
      return -1;
    }
    if (r == ncclSuccess) return 0;
    err = std::string(what) + ": " + ncclGetErrorString(r);
    return -1;
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (bytes == 0) return 0;
    if (aborted) return check(ncclSuccess, "ncclAllGather");
    return check(ncclAllGather(send, recv, bytes, ncclChar, nc, s), "ncclAllGather");
  }
  int allgatherv(const void* send, void* recv, const size_t* counts, const size_t* offs,
                 hipStream_t s) override {
    if (aborted) return check(ncclSuccess, "allgatherv");
    int rc = check(ncclGroupStart(), "ncclGroupStart");
    for (int r = 0; r < world && !rc; ++r) {
      if (counts[r] == 0) continue;
      char* dst = static_cast<char*>(recv) + offs[r];
      rc = check(ncclBroadcast(r == rank ? send : dst, dst, counts[r], ncclChar, r, nc, s),
                 "ncclBroadcast");
    }
    const int rc2 = check(ncclGroupEnd(), "ncclGroupEnd");
    return rc ? rc : rc2;
  }
  int alltoallv(const void* send, const size_t* scnt, const size_t* soff, void* recv,
                const size_t* rcnt, const size_t* roff, hipStream_t s) override {
    if (aborted) return check(ncclSuccess, "alltoallv");
    // the rank's own piece is a local copy
    if (scnt[rank]) {
      if (hipMemcpyAsync(static_cast<char*>(recv) + roff[rank],
                         static_cast<const char*>(send) + soff[rank], scnt[rank],
                         hipMemcpyDeviceToDevice, s) != hipSuccess) {
        err = "alltoallv: local copy";
        return -1;
      }
    }
    int rc = check(ncclGroupStart(), "ncclGroupStart");
    for (int r = 0; r < world && !rc; ++r) {
      if (r == rank) continue;
      if (scnt[r])
        rc = check(ncclSend(static_cast<const char*>(send) + soff[r], scnt[r], ncclChar, r, nc, s),
                   "ncclSend");
      if (!rc && rcnt[r])
        rc = check(ncclRecv(static_cast<char*>(recv) + roff[r], rcnt[r], ncclChar, r, nc, s),
                   "ncclRecv");
    }
    const int rc2 = check(ncclGroupEnd(), "ncclGroupEnd");
    return rc ? rc : rc2;
  }
  int allreduce_min_u32(uint32_t* buf, size_t n, hipStream_t s) override {
    if (n == 0) return 0;
    if (aborted) return check(ncclSuccess, "ncclAllReduce");
    return check(ncclAllReduce(buf, buf, n, ncclUint32, ncclMin, nc, s), "ncclAllReduce");
  }
};

}  // namespace

int rccl_unique_id(void* out128, std::string* err) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    if (err) *err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return -1;
  }
  static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
  memcpy(out128, &id, sizeof(id));
  return 0;
}

Comm* make_rccl_comm(int rank, int world, const void* unique_id, int device, std::string* err) {
  if (hipSetDevice(device) != hipSuccess) {
    if (err) *err = "hipSetDevice";
    return nullptr;
  }
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  auto c = std::make_unique<RcclComm>();
  c->rank = rank;
  c->world = world;
  const ncclResult_t r = ncclCommInitRank(&c->nc, world, id, rank);
  if (r != ncclSuccess) {
    if (err) *err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    c->nc = nullptr;
    return nullptr;
  }
  return c.release();
}

// ===================================================================== in-process group ======
namespace {

struct Hub {
  int world = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;  // a rank failed: every barrier returns at once
  // what each rank posted for the current collective
  std::vector<const void*> ptr;
  std::vector<const size_t*> vec;
  explicit Hub(int w) : world(w), ptr(w, nullptr), vec(w, nullptr) {}
  // false if the group was aborted (by any rank)
  bool barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
    }
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    aborted = true;
    cv.notify_all();
  }
};

struct LocalComm final : Comm {
  std::shared_ptr<Hub> hub;
  uint32_t* tmp = nullptr;  // allreduce scratch
  size_t tmp_n = 0;
  const char* kind() const override { return "local"; }
  ~LocalComm() override {
    if (tmp) (void)hipFree(tmp);
  }
  void abort() override {
    aborted = true;
    hub->abort();
  }
  int sync(hipStream_t s) {
    if (hipStreamSynchronize(s) != hipSuccess) {
      err = "local comm: stream sync";
      return -1;
    }
    return 0;
  }
  int copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return 0;
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s) != hipSuccess) {
      err = "local comm: peer copy";
      return -1;
    }
    return 0;
  }
  // post (p, v), wait for every rank, run body(peer pointers), wait until every rank is done
  // reading before anyone reuses its buffers.
  template <class F>
  int exchange(const void* p, const size_t* v, hipStream_t s, F body) {
    if (int e = sync(s)) return e;  // my send data is complete
    hub->ptr[rank] = p;
    hub->vec[rank] = v;
    if (!hub->barrier()) {
      err = "local comm: group aborted";
      return -1;
    }
    int rc = body();
    if (!rc) rc = sync(s);
    if (!hub->barrier() && !rc) {
      err = "local comm: group aborted";
      rc = -1;
    }
    return rc;
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    return exchange(send, nullptr, s, [&] {
      for (int r = 0; r < world; ++r)
        if (int e = copy(static_cast<char*>(recv) + r * bytes, hub->ptr[r], bytes, s)) return e;
      return 0;
    });
  }
  int allgatherv(const void* send, void* recv, const size_t* counts, const size_t* offs,
                 hipStream_t s) override {
    return exchange(send, nullptr, s, [&] {
      for (int r = 0; r < world; ++r)
        if (int e = copy(static_cast<char*>(recv) + offs[r], hub->ptr[r], counts[r], s)) return e;
      return 0;
    });
  }
  int alltoallv(const void* send, const size_t* scnt, const size_t* soff, void* recv,
                const size_t* rcnt, const size_t* roff, hipStream_t s) override {
    (void)scnt;
    return exchange(send, soff, s, [&] {
      for (int r = 0; r < world; ++r) {
        const char* src = static_cast<const char*>(hub->ptr[r]) + hub->vec[r][rank];
        if (int e = copy(static_cast<char*>(recv) + roff[r], src, rcnt[r], s)) return e;
      }
      return 0;
    });
  }
  int allreduce_min_u32(uint32_t* buf, size_t n, hipStream_t s) override {
    if (tmp_n < 2 * n) {
      if (tmp) (void)hipFree(tmp);
      tmp = nullptr;
      tmp_n = 0;
      if (hipMalloc((void**)&tmp, sizeof(uint32_t) * 2 * std::max<size_t>(n, 1)) != hipSuccess) {
        err = "local comm: scratch";
        return -1;
      }
      tmp_n = 2 * std::max<size_t>(n, 1);
    }
    uint32_t* acc = tmp;
    uint32_t* peer = tmp + n;
    int rc = exchange(buf, nullptr, s, [&] {
      if (int e = copy(acc, buf, 4 * n, s)) return e;
      for (int r = 0; r < world; ++r) {
        if (r == rank) continue;
        if (int e = copy(peer, hub->ptr[r], 4 * n, s)) return e;
        launch_min_u32(acc, peer, n, s);
      }
      return 0;
    });
    if (rc) return rc;
    return copy(buf, acc, 4 * n, s) ? -1 : sync(s);
  }
};

}  // namespace

void make_local_comms(int world, Comm** out) {
  auto hub = std::make_shared<Hub>(world);
  for (int r = 0; r < world; ++r) {
    auto* c = new LocalComm();
    c->rank = r;
    c->world = world;
    c->hub = hub;
    out[r] = c;
  }
}

}  // namespace klsh
