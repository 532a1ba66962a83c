// internal.hpp — shared host-side declarations of libcfd_amd.so.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/cfd_amd.h"

namespace cfd {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

// RCCL transport (comm.hip). Loaded with dlopen on first use so the
// single-GPU library has no RCCL dependency.
struct LoopHub;  // in-process transport (testing the rank path on one device)
struct LoopOp {
  int kind;  // 0 send, 1 recv
  double* buf;
  size_t count;
  int peer;
};

struct Comm {
  void* nccl = nullptr;  // ncclComm_t
  int nranks = 1, rank = 0, device = 0;
  LoopHub* hub = nullptr;  // non-null: loopback transport instead of RCCL
  std::vector<LoopOp> pending;
  void* ev_ready = nullptr;  // hipEvent_t (loopback)
  void* ev_done = nullptr;
  double* tmp = nullptr;     // loopback all-reduce scratch
  size_t tmp_count = 0;
};

void comm_unique_id(unsigned char* id_out);
Comm* comm_init(const unsigned char* id, int nranks, int rank, int device);
LoopHub* loop_hub_create(int nranks);
void loop_hub_destroy(LoopHub* h);
Comm* comm_init_loopback(LoopHub* h, int rank, int device);
void comm_destroy(Comm* c);
void comm_info(Comm* c, int* nranks, int* rank, int* transport);
void comm_group_start(Comm* c);
void comm_group_end(Comm* c, void* stream);
void comm_send(Comm* c, const double* buf, size_t count, int peer, void* stream);
void comm_recv(Comm* c, double* buf, size_t count, int peer, void* stream);
void comm_halo_exchange(Comm* c, const double* send_lo, double* recv_lo, int peer_lo, const double* send_hi,
                        double* recv_hi, int peer_hi, size_t count, void* stream);
long long comm_exchange_check(Comm* c, int peer, size_t count);
void comm_allreduce_max(Comm* c, double* buf, size_t count, void* stream);
void comm_allreduce_sum(Comm* c, double* buf, size_t count, void* stream);

// VTK output (vtk.cpp). Arrays are (ny+2) x (nx+2) row-major host doubles.
void write_vtk_arrays(const cfd_params& p, const std::string& filename, double time_value, const double* uc,
                      const double* vc, const double* pr, const double* temp = nullptr);
void write_pvd(const std::string& filename, const char* const* files, const double* times, int n);

bool host_is_fluid(const cfd_params& p, int j, int i);

}  // namespace cfd
