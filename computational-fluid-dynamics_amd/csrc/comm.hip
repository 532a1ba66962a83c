// comm.hip — RCCL transport for the multi-process strip decomposition.
//
// One process per GPU; each rank owns a strip of rows and exchanges its
// boundary rows with the ranks above and below (point-to-point send/recv over
// xGMI), plus tiny all-reduces for the residual / source maxima and the
// source mean. librccl is dlopen'ed on first use (it resolves to the copy
// already loaded by PyTorch when present, same soname), so single-GPU use of
// libcfd_amd.so never touches RCCL.
#include <dlfcn.h>

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "internal.hpp"

namespace cfd {
namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {
      r.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (r.h) break;
    }
    if (!r.h) return;
    r.GetUniqueId = reinterpret_cast<decltype(r.GetUniqueId)>(dlsym(r.h, "ncclGetUniqueId"));
    r.CommInitRank = reinterpret_cast<decltype(r.CommInitRank)>(dlsym(r.h, "ncclCommInitRank"));
    r.CommDestroy = reinterpret_cast<decltype(r.CommDestroy)>(dlsym(r.h, "ncclCommDestroy"));
    r.GroupStart = reinterpret_cast<decltype(r.GroupStart)>(dlsym(r.h, "ncclGroupStart"));
    r.GroupEnd = reinterpret_cast<decltype(r.GroupEnd)>(dlsym(r.h, "ncclGroupEnd"));
    r.Send = reinterpret_cast<decltype(r.Send)>(dlsym(r.h, "ncclSend"));
    r.Recv = reinterpret_cast<decltype(r.Recv)>(dlsym(r.h, "ncclRecv"));
    r.AllReduce = reinterpret_cast<decltype(r.AllReduce)>(dlsym(r.h, "ncclAllReduce"));
    r.GetErrorString = reinterpret_cast<decltype(r.GetErrorString)>(dlsym(r.h, "ncclGetErrorString"));
    r.CommCount = reinterpret_cast<decltype(r.CommCount)>(dlsym(r.h, "ncclCommCount"));
    r.CommUserRank = reinterpret_cast<decltype(r.CommUserRank)>(dlsym(r.h, "ncclCommUserRank"));
  });
  if (!r.h || !r.GetUniqueId || !r.CommInitRank || !r.Send || !r.Recv || !r.AllReduce || !r.GroupStart ||
      !r.GroupEnd)
    throw Error(CFD_E_COMM, "RCCL (librccl.so.1) could not be loaded");
  return r;
}

void check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess) {
    const char* s = rccl().GetErrorString ? rccl().GetErrorString(e) : "?";
    throw Error(CFD_E_COMM, std::string(what) + ": " + s);
  }
}

}  // namespace

void comm_unique_id(unsigned char* id_out) {
  static_assert(sizeof(ncclUniqueId) <= CFD_COMM_ID_BYTES, "ncclUniqueId larger than CFD_COMM_ID_BYTES");
  ncclUniqueId id;
  check(rccl().GetUniqueId(&id), "ncclGetUniqueId");
  std::memset(id_out, 0, CFD_COMM_ID_BYTES);
  std::memcpy(id_out, &id, sizeof id);
}

Comm* comm_init(const unsigned char* id, int nranks, int rank, int device) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw Error(CFD_E_ARG, "bad rank / nranks");
  if (hipSetDevice(device) != hipSuccess) throw Error(CFD_E_DEVICE, "hipSetDevice failed");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  ncclComm_t c;
  check(rccl().CommInitRank(&c, nranks, uid, rank), "ncclCommInitRank");
  Comm* cm = new Comm;
  cm->nccl = c;
  cm->nranks = nranks;
  cm->rank = rank;
  cm->device = device;
  return cm;
}

void comm_info(Comm* c, int* nranks, int* rank, int* transport) {
  if (!c) throw Error(CFD_E_ARG, "null communicator");
  if (c->hub) {
    *nranks = c->nranks;
    *rank = c->rank;
    *transport = 1;
    return;
  }
  Rccl& r = rccl();
  if (!r.CommCount || !r.CommUserRank) throw Error(CFD_E_COMM, "RCCL lacks ncclCommCount / ncclCommUserRank");
  check(r.CommCount(static_cast<ncclComm_t>(c->nccl), nranks), "ncclCommCount");
  check(r.CommUserRank(static_cast<ncclComm_t>(c->nccl), rank), "ncclCommUserRank");
  *transport = 0;
}

void comm_destroy(Comm* c) {
  if (!c) return;
  if (c->hub) {
    if (c->ev_ready) (void)hipEventDestroy((hipEvent_t)c->ev_ready);
    if (c->ev_done) (void)hipEventDestroy((hipEvent_t)c->ev_done);
    if (c->tmp) (void)hipFree(c->tmp);
  } else if (c->nccl && rccl().CommDestroy) {
    rccl().CommDestroy(static_cast<ncclComm_t>(c->nccl));
  }
  delete c;
}

// ---------------------------------------------------------------- loopback --
// In-process transport with RCCL's semantics for ranks that share one device
// and live in separate host threads of one process (RCCL refuses two ranks on
// one GPU). Only used to test the rank code path; copies are device-to-device
// on the receiving rank's stream, ordered against the sender with events.

constexpr int LOOP_MAX_RANKS = 32;

struct LoopHub {
  int n;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  std::vector<std::vector<LoopOp>> posted;
  std::vector<hipEvent_t> ready, done;
  std::vector<double*> bufs, tmps;
  explicit LoopHub(int nr) : n(nr), posted(nr), ready(nr), done(nr), bufs(nr), tmps(nr) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const long g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

#define LHIP(x)                                                                                     \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw Error(CFD_E_COMM, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

LoopHub* loop_hub_create(int nranks) {
  if (nranks < 1 || nranks > LOOP_MAX_RANKS) throw Error(CFD_E_ARG, "loopback nranks must be in [1, 32]");
  return new LoopHub(nranks);
}
void loop_hub_destroy(LoopHub* h) { delete h; }

Comm* comm_init_loopback(LoopHub* h, int rank, int device) {
  if (!h || rank < 0 || rank >= h->n) throw Error(CFD_E_ARG, "bad loopback rank");
  LHIP(hipSetDevice(device));
  Comm* c = new Comm;
  c->hub = h;
  c->nranks = h->n;
  c->rank = rank;
  c->device = device;
  hipEvent_t a, b;
  LHIP(hipEventCreateWithFlags(&a, hipEventDisableTiming));
  LHIP(hipEventCreateWithFlags(&b, hipEventDisableTiming));
  c->ev_ready = a;
  c->ev_done = b;
  return c;
}

static void loop_group_end(Comm* c, hipStream_t st) {
  LoopHub& h = *c->hub;
  const int me = c->rank;
  LHIP(hipEventRecord((hipEvent_t)c->ev_ready, st));
  h.posted[me] = c->pending;
  h.ready[me] = (hipEvent_t)c->ev_ready;
  h.barrier();
  // receives: copy the matching peer send (k-th send to me from that peer = k-th recv from it)
  for (size_t q = 0; q < c->pending.size(); ++q) {
    const LoopOp& r = c->pending[q];
    if (r.kind != 1) continue;
    int nth = 0;
    for (size_t z = 0; z < q; ++z)
      if (c->pending[z].kind == 1 && c->pending[z].peer == r.peer) ++nth;
    const LoopOp* s = nullptr;
    for (const LoopOp& o : h.posted[r.peer])
      if (o.kind == 0 && o.peer == me && nth-- == 0) { s = &o; break; }
    if (!s || s->count != r.count) throw Error(CFD_E_COMM, "loopback: unmatched send/recv");
    LHIP(hipStreamWaitEvent(st, h.ready[r.peer], 0));
    LHIP(hipMemcpyAsync(r.buf, s->buf, r.count * sizeof(double), hipMemcpyDeviceToDevice, st));
  }
  LHIP(hipEventRecord((hipEvent_t)c->ev_done, st));
  h.done[me] = (hipEvent_t)c->ev_done;
  h.barrier();
  // my send buffers may be overwritten only after the peers' copies
  for (const LoopOp& o : c->pending)
    if (o.kind == 0) LHIP(hipStreamWaitEvent(st, h.done[o.peer], 0));
  h.barrier();
  c->pending.clear();
}

struct LoopPtrs {
  const double* p[LOOP_MAX_RANKS];
};

// Reduction over the ranks' buffers in rank order (a fixed order: every rank
// computes the same bits). The pointer table travels by value in the kernel
// arguments, so the all-reduce is stream-ordered like RCCL's: no host sync.
__global__ void loop_reduce_kernel(LoopPtrs bufs, int n, size_t count, int op, double* out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= count) return;
  double v = bufs.p[0][i];
  for (int r = 1; r < n; ++r) v = op ? fmax(v, bufs.p[r][i]) : v + bufs.p[r][i];
  out[i] = v;
}

static void loop_allreduce(Comm* c, double* buf, size_t count, int op, hipStream_t st) {
  LoopHub& h = *c->hub;
  const int me = c->rank;
  if (c->tmp_count < count) {
    // (a later, larger all-reduce reallocates: drain the stream's uses of the old scratch first)
    if (c->tmp) {
      LHIP(hipStreamSynchronize(st));
      LHIP(hipFree(c->tmp));
    }
    LHIP(hipMalloc(&c->tmp, count * sizeof(double)));
    c->tmp_count = count;
  }
  LHIP(hipEventRecord((hipEvent_t)c->ev_ready, st));
  h.bufs[me] = buf;
  h.ready[me] = (hipEvent_t)c->ev_ready;
  h.barrier();
  for (int r = 0; r < h.n; ++r) LHIP(hipStreamWaitEvent(st, h.ready[r], 0));
  LoopPtrs tab{};
  for (int r = 0; r < h.n; ++r) tab.p[r] = h.bufs[r];
  loop_reduce_kernel<<<(unsigned)((count + 255) / 256), 256, 0, st>>>(tab, h.n, count, op, c->tmp);
  LHIP(hipEventRecord((hipEvent_t)c->ev_done, st));
  h.done[me] = (hipEvent_t)c->ev_done;
  h.barrier();
  for (int r = 0; r < h.n; ++r) LHIP(hipStreamWaitEvent(st, h.done[r], 0));  // all reads of every buf done
  LHIP(hipMemcpyAsync(buf, c->tmp, count * sizeof(double), hipMemcpyDeviceToDevice, st));
  h.barrier();
}

// ----------------------------------------------------------------- dispatch --

void comm_group_start(Comm* c) {
  if (c->hub) { c->pending.clear(); return; }
  check(rccl().GroupStart(), "ncclGroupStart");
}
void comm_group_end(Comm* c, void* stream) {
  if (c->hub) { loop_group_end(c, static_cast<hipStream_t>(stream)); return; }
  check(rccl().GroupEnd(), "ncclGroupEnd");
}

void comm_send(Comm* c, const double* buf, size_t count, int peer, void* stream) {
  if (c->hub) { c->pending.push_back({0, const_cast<double*>(buf), count, peer}); return; }
  check(rccl().Send(buf, count, ncclFloat64, peer, static_cast<ncclComm_t>(c->nccl),
                    static_cast<hipStream_t>(stream)),
        "ncclSend");
}

void comm_recv(Comm* c, double* buf, size_t count, int peer, void* stream) {
  if (c->hub) { c->pending.push_back({1, buf, count, peer}); return; }
  check(rccl().Recv(buf, count, ncclFloat64, peer, static_cast<ncclComm_t>(c->nccl),
                    static_cast<hipStream_t>(stream)),
        "ncclRecv");
}

// The strip decomposition's halo exchange (Solver::exchange): one group of
// send / recv pairs, this rank's rows to the rank below (peer_lo) and above
// (peer_hi) and their rows into this rank's halos; peer < 0: no neighbour.
// Pairs to one peer match in issue order (the peer's first send to this rank
// lands in this rank's first receive from it).
void comm_halo_exchange(Comm* c, const double* send_lo, double* recv_lo, int peer_lo, const double* send_hi,
                        double* recv_hi, int peer_hi, size_t count, void* stream) {
  comm_group_start(c);
  if (peer_lo >= 0) {
    comm_send(c, send_lo, count, peer_lo, stream);
    comm_recv(c, recv_lo, count, peer_lo, stream);
  }
  if (peer_hi >= 0) {
    comm_send(c, send_hi, count, peer_hi, stream);
    comm_recv(c, recv_hi, count, peer_hi, stream);
  }
  comm_group_end(c, stream);
}

// Transport check on device buffers of `count` doubles: both neighbours of the
// halo exchange are `peer` (the rank itself: RCCL's send / recv to self, which
// a one-GPU box can run). Send buffers carry a pattern of (rank, side, index);
// the receives must hold the peer's pattern bit for bit: returns the number of
// mismatching doubles.
long long comm_exchange_check(Comm* c, int peer, size_t count) {
  if (!c) throw Error(CFD_E_ARG, "null communicator");
  if (peer < 0 || peer >= c->nranks) throw Error(CFD_E_ARG, "peer outside the communicator");
  if (count == 0) throw Error(CFD_E_ARG, "count must be > 0");
  LHIP(hipSetDevice(c->device));
  auto pat = [&](int rank, int side, size_t k) { return (double)rank * 1e9 + side * 1e8 + (double)k + 0.375; };
  std::vector<double> h(count);
  double* d[4] = {nullptr, nullptr, nullptr, nullptr};  // send_lo, recv_lo, send_hi, recv_hi
  hipStream_t st = nullptr;
  long long bad = 0;
  try {
    for (double*& x : d) LHIP(hipMalloc(&x, count * sizeof(double)));
    LHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int side = 0; side < 2; ++side) {
      for (size_t k = 0; k < count; ++k) h[k] = pat(c->rank, side, k);
      LHIP(hipMemcpy(d[2 * side], h.data(), count * sizeof(double), hipMemcpyHostToDevice));
      LHIP(hipMemset(d[2 * side + 1], 0xff, count * sizeof(double)));  // (NaN until received)
    }
    comm_halo_exchange(c, d[0], d[1], peer, d[2], d[3], peer, count, st);
    LHIP(hipStreamSynchronize(st));
    for (int side = 0; side < 2; ++side) {
      LHIP(hipMemcpy(h.data(), d[2 * side + 1], count * sizeof(double), hipMemcpyDeviceToHost));
      for (size_t k = 0; k < count; ++k) {
        const double e = pat(peer, side, k);
        if (std::memcmp(&h[k], &e, sizeof e) != 0) ++bad;
      }
    }
  } catch (...) {
    for (double* x : d)
      if (x) (void)hipFree(x);
    if (st) (void)hipStreamDestroy(st);
    throw;
  }
  for (double* x : d) (void)hipFree(x);
  (void)hipStreamDestroy(st);
  return bad;
}

void comm_allreduce_max(Comm* c, double* buf, size_t count, void* stream) {
  if (c->hub) { loop_allreduce(c, buf, count, 1, static_cast<hipStream_t>(stream)); return; }
  check(rccl().AllReduce(buf, buf, count, ncclFloat64, ncclMax, static_cast<ncclComm_t>(c->nccl),
                         static_cast<hipStream_t>(stream)),
        "ncclAllReduce(max)");
}

void comm_allreduce_sum(Comm* c, double* buf, size_t count, void* stream) {
  if (c->hub) { loop_allreduce(c, buf, count, 0, static_cast<hipStream_t>(stream)); return; }
  check(rccl().AllReduce(buf, buf, count, ncclFloat64, ncclSum, static_cast<ncclComm_t>(c->nccl),
                         static_cast<hipStream_t>(stream)),
        "ncclAllReduce(sum)");
}

}  // namespace cfd
