// comm.cpp — RCCL transport for the multi-process strip decomposition.
//
// One process per GPU; each rank owns a strip of rows and exchanges its
// boundary rows with the ranks above and below (point-to-point send/recv over
// xGMI), plus tiny all-reduces for the residual / source maxima and the
// source mean. librccl is dlopen'ed on first use (it resolves to the copy
// already loaded by PyTorch when present, same soname), so single-GPU use of
// libcfd_amd.so never touches RCCL.
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>

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

void comm_destroy(Comm* c) {
  if (!c) return;
  if (c->nccl && rccl().CommDestroy) rccl().CommDestroy(static_cast<ncclComm_t>(c->nccl));
  delete c;
}

void comm_group_start() { check(rccl().GroupStart(), "ncclGroupStart"); }
void comm_group_end() { check(rccl().GroupEnd(), "ncclGroupEnd"); }

void comm_send(Comm* c, const double* buf, size_t count, int peer, void* stream) {
  check(rccl().Send(buf, count, ncclFloat64, peer, static_cast<ncclComm_t>(c->nccl),
                    static_cast<hipStream_t>(stream)),
        "ncclSend");
}

void comm_recv(Comm* c, double* buf, size_t count, int peer, void* stream) {
  check(rccl().Recv(buf, count, ncclFloat64, peer, static_cast<ncclComm_t>(c->nccl),
                    static_cast<hipStream_t>(stream)),
        "ncclRecv");
}

void comm_allreduce_max(Comm* c, double* buf, size_t count, void* stream) {
  check(rccl().AllReduce(buf, buf, count, ncclFloat64, ncclMax, static_cast<ncclComm_t>(c->nccl),
                         static_cast<hipStream_t>(stream)),
        "ncclAllReduce(max)");
}

void comm_allreduce_sum(Comm* c, double* buf, size_t count, void* stream) {
  check(rccl().AllReduce(buf, buf, count, ncclFloat64, ncclSum, static_cast<ncclComm_t>(c->nccl),
                         static_cast<hipStream_t>(stream)),
        "ncclAllReduce(sum)");
}

}  // namespace cfd
