// solver.hip — host orchestration of the MI355X projection solver and the
// C-ABI of libcfd_amd.so (include/cfd_amd.h).
//
// One Solver object = the reference's CavitySolver / ChannelSolver /
// BackwardsStepSolver (cavity-01.cpp:306, channel-01.cpp:284,
// backwards_step-01.cpp:316): device-resident fields, the per-timestep
// methods as kernel launches on one HIP stream, and the SOR loop driven from
// the host with the convergence test evaluated on the device (no host sync
// per iteration). The grid may be split into row strips — several on one
// device (halo copies on the stream) or one per rank (halo rows over RCCL).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "internal.hpp"
#include "kernels.hpp"
#include "lexw.hpp"
#include "small.hpp"
#include "tile.hpp"
#include "resident.hpp"
#include "open.hpp"
#include "smlex.hpp"
#include "seqsum.hpp"

// 1: the reference order's ramp launches march the wall column tiles as two
// half bands each (lexw.hpp LexRamp::wsplit): the wall tiles' masked march set
// the ramp launches' time (per-launch stamps); cavity 4096^2 704-717 -> 717-729
// GLUPS, channel and 1024^2 neutral to +0.5 % (profiles/r4_lexw_stamps)
#ifndef CFD_LEXW_WALL_SPLIT
#define CFD_LEXW_WALL_SPLIT 1
#endif

namespace cfd {

static thread_local std::string g_last_error;
void set_last_error(const std::string& m) { g_last_error = m; }

#define HIPC(x)                                                                                  \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) throw Error(CFD_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(CFD_E_DEVICE, std::string("launch ") + what + ": " + hipGetErrorString(e));
}

enum { B_P0 = 0, B_P1, B_F, B_US, B_VS, B_U, B_V, B_UC, B_VC, B_PL, B_P2, B_T, B_T2, NB };  // B_T/B_T2: Rayleigh-Benard only;  // B_PL: lex-mode initial field;
// B_P2: third pressure buffer of the lagged convergence test (ranks)
static int pbuf(int idx) { return idx == 0 ? B_P0 : idx == 1 ? B_P1 : B_P2; }

constexpr int MARCH_MIN_TH = 24;   // minimum rows per band of a wave-march launch
constexpr int OVL_ROWS = 16;       // rows next to each neighbour updated by the overlapped boundary launch

struct Strip {
  Geo g{};
  double* b[NB] = {};
  dim3 grid2d;          // 64 x 4 blocks over owned interior rows
  size_t part_off = 0;  // offset into the partial-sum buffer
};

static Coef make_coef(const cfd_params& p) {
  Coef c{};
  c.case_id = p.case_id;
  c.step_i = p.step_i;
  c.inlet_jmax = p.inlet_jmax;
  c.dx = p.dx;
  c.dy = p.dy;
  c.idx = 1.0 / p.dx;
  c.idy = 1.0 / p.dy;
  c.idx2 = 1.0 / (p.dx * p.dx);
  c.idy2 = 1.0 / (p.dy * p.dy);
  c.nu = p.nu;
  c.dt = p.dt;
  c.rho = p.rho;
  c.u_ref = p.u_ref;
  c.omega = p.omega;
  c.one_m_omega = 1.0 - p.omega;
  for (int n = 0; n < 5; ++n) c.om_nc[n] = (n > 0) ? p.omega / n : 0.0;
  c.h2 = p.dx * p.dx;
  c.denom = 2.0 * (c.idx2 + c.idy2);
  c.rdenom = 1.0 / c.denom;
  c.rdenom_lo = std::fma(-c.rdenom, c.denom, 1.0) / c.denom;  // (device.hpp div_denom)
  c.cav_src = (1.0 / p.dt) * p.rho;
  c.open_src = p.rho / p.dt;
  c.cav_corr = (p.dt / p.dx) * p.rho;
  c.open_cu = p.dt / (p.rho * p.dx);
  c.open_cv = p.dt / (p.rho * p.dy);
  c.tol_factor = p.tol_factor;
  c.abs_tol = p.abs_tol;
  // proof-mode test (kernels.hpp, proof_ratio): its error bound assumes
  // 1 - omega and omega / 4 exact, i.e. 0.5 <= omega <= 2
  const bool open = p.case_id == CFD_CHANNEL || p.case_id == CFD_BACKSTEP;
  c.proof_k = (p.omega >= 0.5 && p.omega < 2.0 && p.omega != 1.0)
                  ? (open ? c.denom : 4.0 * c.idx2) * std::fabs(1.0 - p.omega) / p.omega
                  : 0.0;
  c.proof_pm = open ? c.denom : c.idx2;
  c.proof_fd = open ? c.rdenom * (1.0 + 0x1p-50) : c.h2;
  c.kappa = p.kappa;
  c.buoy = p.buoyancy;
  c.t_hot = p.t_hot;
  c.t_cold = p.t_cold;
  c.t_ref = p.t_ref;
  return c;
}

class Solver {
 public:
  cfd_params P{};
  Coef C{};
  int dev = 0;
  hipStream_t st = nullptr;
  std::vector<Strip> S;
  Comm* comm = nullptr;  // non-null: this process is one rank of a strip decomposition
  int pcur = 0;          // which p buffer (pbuf index) holds the current pressure
  int pitch = 0;
  double fluid_count = 0;

  double *ring = nullptr, *srcmax = nullptr, *divmax = nullptr, *tolv = nullptr, *partials = nullptr,
         *total = nullptr;
  int* stop = nullptr;
  void* seqws = nullptr;  // seq_sum_launch's chunk records (seqsum.hip)
  size_t seqws_bytes = 0;
  int* seqcnt = nullptr;  // chunks the sequential sums ran as the plain chain (device counter)
  size_t npart = 0;
  int* h_stat = nullptr;    // pinned: 2 x {stop, iter}
  double* h_shard = nullptr;  // pinned: RES_SHARDS*SHARD_STRIDE
  hipEvent_t ev_poll[2] = {}, ev_a = nullptr, ev_b = nullptr;
  hipEvent_t ev_s0 = nullptr, ev_s1 = nullptr;  // around the last whole timestep (cfd_timing.step_ms)
  bool step_timed = false;                      // ev_s0/ev_s1 hold a step not yet added to T.step_ms
  // Halo overlap on ranks (RCCL): the rows next to the neighbours and the
  // exchange run on st_b while the interior rows run on st.
  hipStream_t st_b = nullptr;
  hipEvent_t ev_int[2] = {}, ev_bnd[2] = {}, ev_sync = nullptr;
  bool overlap = false;     // enabled for ranks with enough rows (cfd_params.overlap = CFD_OFF disables)
  // With overlap the convergence test lags one more pair: launch m tests the
  // residuals of pair m-2, whose all-reduce then runs beside launch m-1
  // instead of in front of launch m. A third pressure buffer keeps the input
  // and output of the pair a late stop lands in intact.
  bool lagged() const { return overlap && sweeps_per_launch() >= 2; }
  // red-black iterations per exact-residual SOR launch: 3 for the cavity (its
  // depth-7 pipeline fits the 8-row halos), 2 for the open cases, 1 or 2 on
  // request (proof-mode launches: proof_ns)
  int sweeps_per_launch() const {
    if (tile_on) {  // LDS-tile launches: any count up to what the halo covers
      const int mx = tile_max_sweeps(P.case_id);
      return (P.sweeps_per_launch >= 1 && P.sweeps_per_launch < mx) ? P.sweeps_per_launch : mx;
    }
    if (P.sweeps_per_launch == 1) return 1;
    if (P.sweeps_per_launch == 2) return 2;
    return P.case_id == CFD_CAVITY ? 3 : 2;
  }
  // LDS-tile launches (tile.hpp): red-black, one strip, no ranks, a grid of at
  // most tile_rounds resident rounds of tiles (CFD_TUNE_TILE_ROUNDS). Default:
  // 1 for the cavity, 0 for the open cases (their wave march with unchecked
  // row groups is faster: channel 4096x512 8.2 us per sweep against 9.9)
  bool tile_on = false;
  int tile_rounds = 1;  // (open cases: 0, set in init)
  TilePlan tplan{};
  void plan_tiles() {
    tile_on = false;
    tplan = TilePlan{};
    if (P.ordering != CFD_ORDER_RB || S.size() != 1 || comm || tile_rounds <= 0) return;
    const Geo& g = S[0].g;
    tplan = tile_plan(P.nx, g.wj0, g.wj1 + 1, tile_rounds * n_cu);
    tile_on = tplan.ctiles > 0;
  }
  // Register-resident whole-solve launch (resident.hpp): the cavity and the
  // channel, one strip, no ranks, both orders (red-black with proof mode), a
  // grid of at most one tile per CU whose tiles can all be resident at once
  // (the occupancy of the kernel instance: its workgroups wait on each other)
  // (CFD_TUNE_RESIDENT). Its exchange fields and state words are allocated at
  // the first solve.
  bool res_knob = false;
  bool res_on = false;
  ResPlan rplan{};
  double* res_x[2] = {nullptr, nullptr};
  unsigned* res_state = nullptr;
  size_t res_state_n = 0;
  // (the reference order too: resident.hip's LEX kernel, sampled exceedance
  // bits instead of the proof; the reference-sized grids keep smlex.hip)
  unsigned long long* res_bits = nullptr;
  size_t res_bits_n = 0;
  void plan_resident() {
    res_on = false;
    rplan = ResPlan{};
    if (!res_knob || S.size() != 1 || comm || thermal) return;
    // the cavity and the channel, both orders
    const bool open = P.case_id == CFD_CHANNEL;
    if (P.case_id != CFD_CAVITY && !open) return;
    if (P.ordering == CFD_ORDER_RB && (!proof_enabled || !(C.proof_k > 0.0))) return;
    const Geo& g = S[0].g;
    rplan = res_plan(P.nx, g.wj0, g.wj1 + 1, n_cu, open, P.ordering == CFD_ORDER_LEX);
    res_on = rplan.ctiles > 0 &&
             rplan.ctiles * rplan.rtiles <= res_coresident_tiles(open ? CHANNEL : CAVITY, P.ordering == CFD_ORDER_LEX,
                                                                 rplan, n_cu);
  }
  struct LaunchRec {
    int first, n;        // iterations first .. first+n-1
    bool proof = false;  // its ring slots hold proof ratios (proof-mode launch), not residuals
  };
  // Proof-mode convergence test (kernels.hpp, proof_ratio): cavity 3-sweep
  // launches prove "the reference goes on" from the black updates instead of
  // evaluating the residual; an iteration it leaves open is evaluated exactly
  // (the solve falls back to exact launches from the launch that computed it).
  bool proof_launch = false;  // the launch being enqueued runs in proof mode
  bool window_proof = false;  // the window it tests was computed in proof mode
  bool proof_enabled = true;  // cfd_params.proof_test = CFD_OFF: exact residuals throughout
  int proof_ns = 4;           // sweeps per proof-mode launch (4; 3 with sweeps_per_launch = 3)
  bool proof_ok() const {
    // (only interior column tiles prove: at least one between the two boundary tiles)
    if (tile_on) return proof_enabled && C.proof_k > 0.0;  // tile launches: every case (tile.hip)
    // march launches: the cavity's 3-sweep plan or the open cases' pairs
    // become 4-sweep proof launches (open cases: open.hip)
    const bool plan = P.case_id == CFD_CAVITY ? sweeps_per_launch() == 3
                                              : (P.sweeps_per_launch == 0 || P.sweeps_per_launch == 4);
    return proof_enabled && plan && C.proof_k > 0.0 &&
           (P.nx + 2 + PAIR_TWC - 1) / PAIR_TWC >= 3;
  }
  std::vector<LaunchRec> launches;  // SOR launches of the current solve
  LaunchRec ar_pending{0, 0};       // overlapped launch whose residual all-reduce is not enqueued yet

  // enqueue the pending (lagged) all-reduce of an overlapped launch on xs
  void flush_allreduce(hipStream_t xs) {
    if (ar_pending.n > 0) allreduce_slots(ar_pending.first, ar_pending.n, xs);
    ar_pending = {0, 0};
  }
  int nbufs() const { return lagged() ? 3 : 2; }
  bool b_pending = false;   // st_b has work that st has not waited for yet
  int last_bnd = 0;         // ev_bnd slot recorded last
  long long n_overlapped = 0;  // overlapped pair launches enqueued (this solve)
  cfd_timing T{};
  int resident_waves = 2048;  // wave-march tiles in flight (CUs x 4 SIMDs x waves per SIMD)
  int resident_pair_waves = 2048;  // the same for the two-iteration kernel
  int pair_edge_pct = 45;          // boundary-column band length, % of the interior march (open cases; cavity: 80)
  int march_flags = 3;         // bit 0 alternate directions, bit 1 XCD-aware order, bit 3 column-major tile order
  int march_min_th = MARCH_MIN_TH;
  int tent_th = 64;            // rows per band of the predictor's march
  int n_cu = 256;              // compute units of the device

  // cfd_set_tuning (include/cfd_amd.h enum cfd_tuning): launch planning only
  void set_tuning(int knob, int v) {
    set_tuning_value(knob, v);
    if (knob == CFD_TUNE_TILE_ROUNDS) plan_tiles();
    if (knob == CFD_TUNE_RESIDENT) plan_resident();
  }
  void set_tuning_value(int knob, int v) {
    switch (knob) {
      case CFD_TUNE_PAIR_WPS: resident_pair_waves = std::max(1, std::min(v, 4)) * 4 * n_cu; break;
      case CFD_TUNE_WAVE_WPS: resident_waves = std::max(1, std::min(v, 4)) * 4 * n_cu; break;
      case CFD_TUNE_LEXW_WAVES: resident_lexw_waves = std::max(64, v); break;
      case CFD_TUNE_LEXW_EDGE_PCT: lexw_edge_pct = std::max(10, std::min(100, v)); break;
      case CFD_TUNE_PAIR_EDGE_PCT: pair_edge_pct = std::max(10, std::min(100, v)); break;
      case CFD_TUNE_MARCH_MIN_TH: march_min_th = std::max(1, v); break;
      case CFD_TUNE_TENT_TH: tent_th = std::max(4, v); break;
      case CFD_TUNE_LEXW_RAMP_PCT: lexw_ramp_pct = std::max(0, std::min(100, v)); break;
      case CFD_TUNE_TILE_ROUNDS: tile_rounds = std::max(0, std::min(v, 16)); break;
      case CFD_TUNE_MARCH_ORDER: march_flags = (march_flags & ~8) | (v ? 8 : 0); break;
      case CFD_TUNE_LEXW_LEFT: lexw_left = v != 0; break;
      case CFD_TUNE_RESIDENT: res_knob = v != 0; break;
      case CFD_TUNE_LEXW_UPDOWN: lexw_updown = v != 0; break;
      default: throw Error(CFD_E_ARG, "unknown tuning knob");
    }
  }

  // The reference's lexicographic order at any size (lexw.hpp): per-slot
  // exceedance bitset, final-residual shards, events around the steady-state
  // launches (no ramp), resident waves of the lexw kernel.
  unsigned long long* lexbits = nullptr;
  size_t lexbits_words = 0;
  double* resmax = nullptr;
  hipEvent_t ev_f0 = nullptr, ev_f1 = nullptr;
  int resident_lexw_waves = 2048;
  int lexw_edge_pct = 100;  // wall-tile band length, % of the interior band (cfd_tuning_default: 75 up to 2048 rows)
  int lexw_ramp_pct = 0;    // ramp launches: bands at least this % of the steady plan's (CFD_TUNE_LEXW_RAMP_PCT)
  bool lexw_left = true;    // backwards step: the left column tiles' class (CFD_TUNE_LEXW_LEFT)
  bool lexw_updown = true;  // cavity steady launches: odd interior bands march up (CFD_TUNE_LEXW_UPDOWN)
  // the multi-block reference-order march (lexw.hpp): cavity (1-4 sweeps per
  // launch), channel and backwards step (4; 3 on strips). The step's solid
  // rules need a block of at least 2 columns and 2 rows (si >= 2, jb <= ny-1);
  // other step geometries keep the one-workgroup kernel (poisson_lex_kernel)
  bool step_lexw_ok() const { return P.step_i >= 2 && P.inlet_jmax >= 1 && P.inlet_jmax <= P.ny - 2; }
  bool use_lexw() const {
    return P.ordering == CFD_ORDER_LEX &&
           (P.case_id == CFD_CAVITY || P.case_id == CFD_CHANNEL || (P.case_id == CFD_BACKSTEP && step_lexw_ok()));
  }
  double* cscr = nullptr;  // the step's deferred corner residual across launches (LexCtl::cscr)
  // sweeps per reference-order launch: 4 (auto) on one strip; strips and
  // ranks keep 3 (their 8-row halos serve up to 3, lexw.hpp lexw_twc); the
  // cavity also 1-3
  int lexw_ns() const {
    const int ns = (P.case_id != CFD_CAVITY || P.sweeps_per_launch < 1) ? 4 : P.sweeps_per_launch;
    return multi() ? std::min(ns, 3) : ns;
  }
  bool ranks() const { return comm && comm->nranks > 1; }
  // Reference order on ranks: the exceedance bits of the iterations every
  // cell has contributed to are OR-ed over the ranks (lexw_bits_gather /
  // scatter around a max all-reduce) every LEXW_RED_EVERY launches, before the
  // launches that test them; a stop found up to that many launches late costs
  // nothing but those launches (a stop is replayed from the initial field).
  static constexpr int LEXW_RED_EVERY = 8;
  double* lexflags = nullptr;  // K + 1 doubles: the all-reduced bits
  size_t lexflags_n = 0;
  void lexw_reduce_bits(const LexCtl& L, int ka, int kb) {
    if (!ranks() || ka > kb) return;
    const int n = kb - ka + 1;
    if ((size_t)n > lexflags_n) throw Error(CFD_E_STATE, "lexicographic ordering: bit reduction range");
    lexw_bits_gather_kernel<<<(n + 255) / 256, 256, 0, st>>>(L, ka, kb, lexflags);
    check_launch("lexw_bits_gather");
    comm_allreduce_max(comm, lexflags, (size_t)n, st);
    lexw_bits_scatter_kernel<<<(n + 255) / 256, 256, 0, st>>>(L, ka, kb, lexflags);
    check_launch("lexw_bits_scatter");
  }
  // The reference order's sequential sums on ranks (the open cases' source
  // sum, channel-01.cpp:620-628 / backwards_step-01.cpp:843-862, and the
  // kinetic energy of the statistics, cavity-01.cpp:750-755): one chain of
  // dependent adds in the reference's loop order (rows ascending). Ranks own
  // consecutive row blocks in rank order, so rank r continues from rank r-1's
  // running sum (a one-double send / recv per link) and the last rank's
  // total goes back to every rank: the same bits as one device. Every rank
  // issues the same group sequence (the loopback transport needs it; RCCL
  // takes the empty groups as no-ops).
  void seq_sum(const Strip& s, const double* a, const double* b, int mode, double* acc, bool accumulate) {
    T.seqsum_chunks += seq_sum_launch(s.g, C, a, b, mode, acc, accumulate ? 1 : 0, seqws, seqws_bytes, seqcnt, st);
    check_launch("seq_sum");
  }
  // the device counter of plain-chain chunks into T (and back to zero)
  void flush_seq_count() {
    int n = 0;
    HIPC(hipMemcpyAsync(&n, seqcnt, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPC(hipMemsetAsync(seqcnt, 0, sizeof(int), st));
    HIPC(hipStreamSynchronize(st));
    T.seqsum_serial_chunks += n;
  }
  void seq_sum_ranks(int a, int b, int mode, double* acc) {
    const int R = comm->nranks, me = comm->rank;
    const Strip& s = S[0];
    for (int q = 0; q < R; ++q) {
      if (q == me) seq_sum(s, s.b[a], b >= 0 ? s.b[b] : nullptr, mode, acc, me > 0);
      if (q + 1 < R) {
        comm_group_start(comm);
        if (me == q) comm_send(comm, acc, 1, q + 1, st);
        if (me == q + 1) comm_recv(comm, acc, 1, q, st);
        comm_group_end(comm, st);
      }
    }
    comm_group_start(comm);
    if (me == R - 1) {
      for (int p = 0; p < R - 1; ++p) comm_send(comm, acc, 1, p, st);
    } else {
      comm_recv(comm, acc, 1, R - 1, st);
    }
    comm_group_end(comm, st);
  }
  // rows one lexw wave marches beyond its band: the pipeline (2NS+1 each side) + parity row
  static int lexw_extra(int ns) { return 2 * (2 * ns + 1) + 1; }

  // Rayleigh-Benard: the cavity's projection (P.case_id is set to CFD_CAVITY,
  // u_ref 0 = lid at rest) plus the temperature stage on tcur/tnext.
  bool thermal = false;
  int tcur = B_T, tnext = B_T2;

  Solver(const cfd_params& p, int device, const std::vector<std::pair<int, int>>& rows, Comm* cm)
      : P(p), dev(device), comm(cm) {
    try {
      init(rows);
    } catch (...) {
      release();  // whatever the failed construction allocated so far
      throw;
    }
  }

  void init(const std::vector<std::pair<int, int>>& rows) {
    if (P.case_id == CFD_RAYLEIGH_BENARD) {
      thermal = true;
      if (!(P.kappa > 0)) throw Error(CFD_E_ARG, "Rayleigh-Benard needs kappa > 0");
      if (std::fabs(P.dx - P.dy) > 1e-12 * P.dx) throw Error(CFD_E_ARG, "Rayleigh-Benard needs dx == dy");
      P.case_id = CFD_CAVITY;
      P.u_ref = 0.0;
    }
    validate((int)rows.size());
    C = make_coef(P);
    proof_enabled = P.proof_test != CFD_OFF;
    proof_ns = P.sweeps_per_launch == 3 ? 3 : 4;
    HIPC(hipSetDevice(dev));
    hipDeviceProp_t prop;
    HIPC(hipGetDeviceProperties(&prop, dev));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      throw Error(CFD_E_DEVICE, std::string("libcfd_amd requires gfx950 (MI355X); device is ") + prop.gcnArchName);
    HIPC(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    n_cu = prop.multiProcessorCount;
    {
      int wps = 0;  // waves per SIMD of the wave-march kernel (1 block of 4 waves = 1 wave per SIMD)
      HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&wps, poisson_wave_kernel<CAVITY>, 256, 0));
      wps = std::max(1, std::min(wps, 4));
      resident_waves = wps * 4 * prop.multiProcessorCount;
      int pps = 0;
      if (P.case_id == CFD_CAVITY)  // resident waves of the launch the solve runs most
        HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pps, poisson_multi_kernel<CAVITY, 3>, 256, 0));
      else if (P.case_id == CFD_CHANNEL)
        HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pps, poisson_multi_kernel<CHANNEL, 2>, 256, 0));
      else
        HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pps, poisson_multi_kernel<BACKSTEP, 2>, 256, 0));
      pps = std::max(1, std::min(pps, 4));
      // device-independent plan defaults (params.cpp cfd_tuning_default):
      // cavity boundary-column bands 80 % of the interior march (lane-constant
      // indicators), the open cases 45 %; band floor 16 rows for the channel
      // and the reference order, 24 for the red-black cavity / step; LDS tiles
      // for the cavity only
      for (int knob : {CFD_TUNE_LEXW_EDGE_PCT, CFD_TUNE_PAIR_EDGE_PCT, CFD_TUNE_MARCH_MIN_TH, CFD_TUNE_TENT_TH,
                       CFD_TUNE_LEXW_RAMP_PCT, CFD_TUNE_TILE_ROUNDS, CFD_TUNE_MARCH_ORDER, CFD_TUNE_LEXW_LEFT,
                       CFD_TUNE_RESIDENT, CFD_TUNE_LEXW_UPDOWN}) {
        int v = 0;
        if (cfd_tuning_default(&P, knob, &v) == CFD_OK) set_tuning_value(knob, v);
      }
      // cavity proof-mode launches planned for 2 waves per SIMD (taller
      // bands: fewer halo rows), exact ones for 3 (measured at 4096^2, §4)
      if (P.case_id == CFD_CAVITY && proof_ok()) pps = std::min(pps, 2);
      if (use_lexw()) {
        int lps = 0;
        if (P.case_id == CFD_CHANNEL)
          HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&lps, poisson_lexw_kernel<CHANNEL, 4, false, true>, 256, 0));
        else if (P.case_id == CFD_BACKSTEP)
          HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&lps, poisson_lexw_kernel<BACKSTEP, 4, false, true>, 256, 0));
        else if (lexw_ns() == 4)
          HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&lps, poisson_lexw_kernel<CAVITY, 4, false, true>, 256, 0));
        else if (lexw_ns() == 1)
          HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&lps, poisson_lexw_kernel<CAVITY, 1, false>, 256, 0));
        else if (lexw_ns() == 2)
          HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&lps, poisson_lexw_kernel<CAVITY, 2, false>, 256, 0));
        else
          HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&lps, poisson_lexw_kernel<CAVITY, 3, false, true>, 256, 0));
        resident_lexw_waves = std::max(1, std::min(lps, 4)) * 4 * prop.multiProcessorCount;
      }
      resident_pair_waves = pps * 4 * prop.multiProcessorCount;
    }
    pitch = ((P.nx + 3) + 15) / 16 * 16;  // >= nx+3: column pairs (gi, gi+1) stay inside a row
    size_t part = 0;
    for (auto [j0, j1] : rows) {
      S.emplace_back();  // owned by the solver before its buffers exist (release() frees them)
      Strip& s = S.back();
      Geo& g = s.g;
      g.nx = P.nx;
      g.ny = P.ny;
      g.pitch = pitch;
      g.j0 = j0;
      g.j1 = j1;
      g.wj0 = (j0 == 1) ? 0 : j0;
      g.wj1 = (j1 == P.ny) ? P.ny + 1 : j1;
      g.row_lo = j0 - HALO;
      g.nrows = (j1 - j0 + 1) + 2 * HALO;
      const size_t n = (size_t)g.nrows * (size_t)pitch;
      for (int k = 0; k < NB; ++k) {
        if ((k == B_T || k == B_T2) && !thermal) continue;
        HIPC(hipMalloc(&s.b[k], n * sizeof(double)));
        HIPC(hipMemsetAsync(s.b[k], 0, n * sizeof(double), st));
      }
      s.grid2d = dim3((P.nx + 2 + 63) / 64, (j1 - j0 + 1 + 3) / 4);
      s.part_off = part;
      part += (size_t)s.grid2d.x * s.grid2d.y;
    }
    npart = part;
    const size_t ringn = (size_t)RING * RES_SHARDS * SHARD_STRIDE;
    HIPC(hipMalloc(&ring, ringn * sizeof(double)));
    HIPC(hipMalloc(&srcmax, RES_SHARDS * SHARD_STRIDE * sizeof(double)));
    HIPC(hipMalloc(&divmax, RES_SHARDS * SHARD_STRIDE * sizeof(double)));
    HIPC(hipMalloc(&tolv, 4 * sizeof(double)));
    HIPC(hipMalloc(&total, 4 * sizeof(double)));
    HIPC(hipMalloc(&partials, std::max<size_t>(npart, 1) * sizeof(double)));
    HIPC(hipMalloc(&stop, 2 * sizeof(int)));
    HIPC(hipMalloc(&resmax, RES_SHARDS * SHARD_STRIDE * sizeof(double)));
    HIPC(hipMalloc(&cscr, 4 * sizeof(double)));
    long long terms = 1;
    for (auto& s : S) terms = std::max(terms, (long long)(std::min(s.g.j1, P.ny) - std::max(s.g.j0, 1) + 1) * P.nx);
    seqws_bytes = seq_sum_workspace(terms);
    HIPC(hipMalloc(&seqws, seqws_bytes));
    HIPC(hipMalloc(&seqcnt, 8 * sizeof(int)));  // [0] the count ([1..5]: CFD_SEQ_STAMPS builds' phase ticks)
    HIPC(hipMemsetAsync(seqcnt, 0, 8 * sizeof(int), st));
    HIPC(hipMemsetAsync(ring, 0, ringn * sizeof(double), st));
    HIPC(hipMemsetAsync(tolv, 0, 4 * sizeof(double), st));
    HIPC(hipMemsetAsync(stop, 0, 2 * sizeof(int), st));
    HIPC(hipHostMalloc(&h_stat, 4 * sizeof(int), hipHostMallocDefault));
    HIPC(hipHostMalloc(&h_shard, RES_SHARDS * SHARD_STRIDE * sizeof(double), hipHostMallocDefault));
    for (auto& e : ev_poll) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPC(hipEventCreate(&ev_a));
    HIPC(hipEventCreate(&ev_b));
    HIPC(hipEventCreate(&ev_s0));
    HIPC(hipEventCreate(&ev_s1));
    HIPC(hipEventCreate(&ev_f0));
    HIPC(hipEventCreate(&ev_f1));
    if (comm && comm->nranks > 1 && S.size() == 1) {
      const Geo& g0 = S[0].g;
      overlap = P.overlap != CFD_OFF && (g0.wj1 - g0.wj0 + 1) >= 3 * OVL_ROWS;
      if (overlap) {
        HIPC(hipStreamCreateWithFlags(&st_b, hipStreamNonBlocking));
        for (int q = 0; q < 2; ++q) {
          HIPC(hipEventCreateWithFlags(&ev_int[q], hipEventDisableTiming));
          HIPC(hipEventCreateWithFlags(&ev_bnd[q], hipEventDisableTiming));
        }
        HIPC(hipEventCreateWithFlags(&ev_sync, hipEventDisableTiming));
      }
    }
    plan_tiles();
    plan_resident();
    // the step's proof launches on strips / ranks: 3 sweeps (open.hip: its
    // block edge reads one row deeper than the 4-sweep pipeline's 8)
    if (P.case_id == CFD_BACKSTEP && multi()) proof_ns = 3;
    // fluid cells (backwards_step-01.cpp:522-528)
    long long solid = 0;
    if (P.case_id == CFD_BACKSTEP)
      solid = (long long)std::min(P.step_i, P.nx) * (long long)std::max(0, P.ny - P.inlet_jmax);
    fluid_count = (double)((long long)P.nx * P.ny - solid);
    // channel-01.cpp:352 / backwards_step-01.cpp:396: constructor applies the velocity BCs
    if (P.case_id != CFD_CAVITY) apply_bc(false);
    if (thermal) init_temperature();
    HIPC(hipStreamSynchronize(st));
  }

  // Initial temperature (oracle/cfd_oracle.c orc_create): conduction profile
  // plus one roll's perturbation, set on the host once like the reference's
  // field initialisation, then uploaded.
  void init_temperature() {
    int rows, cols, first, last;
    field_dims(CFD_FIELD_T, rows, cols);
    owned_field_rows(CFD_FIELD_T, first, last);
    std::vector<double> h((size_t)(last - first + 1) * cols, 0.0);
    const double pi = 3.14159265358979323846;
    const double length = P.length;
    for (int j = std::max(first, 1); j <= std::min(last, P.ny); ++j)
      for (int i = 1; i <= P.nx; ++i) {
        const double x = (i - 0.5) * P.dx, y = (j - 0.5) * P.dy;
        h[(size_t)(j - first) * cols + i] =
            P.t_hot + (P.t_cold - P.t_hot) * y + P.t_perturb * std::sin(pi * y) * std::cos(pi * x / length);
      }
    transfer(CFD_FIELD_T, nullptr, h.data(), h.size());
  }

  // Rayleigh-Benard stage (oracle orc_temperature_bc + orc_thermal): ghosts,
  // halo rows, then the fused buoyancy + advection-diffusion kernel. Needs the
  // u/v halos compute_tentative() exchanged.
  void advance_temperature() {
    if (!thermal) throw Error(CFD_E_STATE, "cfd_advance_temperature: not a Rayleigh-Benard solver");
    for (auto& s : S) {
      const int n = std::max(P.nx, s.g.j1 - s.g.j0 + 1);
      bc_temperature_kernel<<<(n + 255) / 256, 256, 0, st>>>(s.g, C, s.b[tcur]);
      check_launch("bc_temperature");
    }
    if (multi()) exchange(tcur, 1);
    for (auto& s : S) {
      thermal_kernel<<<s.grid2d, 256, 0, st>>>(s.g, C, s.b[B_U], s.b[B_V], s.b[tcur], s.b[tnext], s.b[B_VS]);
      check_launch("thermal");
    }
    std::swap(tcur, tnext);
  }

  ~Solver() { release(); }

  // Frees everything; both streams are drained before any buffer they may
  // still touch is released. Safe on a partly constructed solver.
  void release() noexcept {
    (void)hipSetDevice(dev);
    if (st_b) (void)hipStreamSynchronize(st_b);
    if (st) (void)hipStreamSynchronize(st);
    for (auto& s : S)
      for (auto* p : s.b)
        if (p) (void)hipFree(p);
    S.clear();
    for (double* p : {ring, srcmax, divmax, tolv, total, partials, resmax, cscr})
      if (p) (void)hipFree(p);
    ring = srcmax = divmax = tolv = total = partials = resmax = cscr = nullptr;
    if (seqws) (void)hipFree(seqws);
    if (seqcnt) (void)hipFree(seqcnt);
    seqws = nullptr;
    seqcnt = nullptr;
    if (lexbits) (void)hipFree(lexbits);
    lexbits = nullptr;
    if (lexflags) (void)hipFree(lexflags);
    lexflags = nullptr;
    lexflags_n = 0;
    if (smlex_ck) (void)hipFree(smlex_ck);
    smlex_ck = nullptr;
    for (auto*& x : res_x) {
      if (x) (void)hipFree(x);
      x = nullptr;
    }
    if (res_state) (void)hipFree(res_state);
    res_state = nullptr;
    res_state_n = 0;
    if (res_bits) (void)hipFree(res_bits);
    res_bits = nullptr;
    res_bits_n = 0;
    lexbits_words = 0;
    if (stop) (void)hipFree(stop);
    stop = nullptr;
    if (h_stat) (void)hipHostFree(h_stat);
    if (h_shard) (void)hipHostFree(h_shard);
    h_stat = nullptr;
    h_shard = nullptr;
    for (auto& e : ev_poll)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ev_a, ev_b, ev_s0, ev_s1, ev_f0, ev_f1})
      if (e) (void)hipEventDestroy(e);
    for (int q = 0; q < 2; ++q) {
      if (ev_int[q]) (void)hipEventDestroy(ev_int[q]);
      if (ev_bnd[q]) (void)hipEventDestroy(ev_bnd[q]);
    }
    if (ev_sync) (void)hipEventDestroy(ev_sync);
    if (st_b) (void)hipStreamDestroy(st_b);
    if (st) (void)hipStreamDestroy(st);
    ev_poll[0] = ev_poll[1] = ev_a = ev_b = ev_s0 = ev_s1 = ev_f0 = ev_f1 = ev_sync = nullptr;
    ev_int[0] = ev_int[1] = ev_bnd[0] = ev_bnd[1] = nullptr;
    st = st_b = nullptr;
  }

  void validate(int nstrips) const {
    if (P.case_id < 0 || P.case_id > 2) throw Error(CFD_E_ARG, "unknown case_id");
    if (P.nx < 2 || P.ny < 2) throw Error(CFD_E_ARG, "grid must have at least 2 interior cells per direction");
    if (!(P.dx > 0) || !(P.dy > 0) || !(P.dt > 0) || !(P.nu > 0) || !(P.rho > 0))
      throw Error(CFD_E_ARG, "dx, dy, dt, nu and rho must be positive");
    if (!(P.omega > 0) || !(P.omega < 2)) throw Error(CFD_E_ARG, "SOR omega must lie in (0, 2)");
    if (P.max_iters < 0) throw Error(CFD_E_ARG, "max_iters must be >= 0");
    if (P.check_every < 1) throw Error(CFD_E_ARG, "check_every must be >= 1");
    if (P.sweeps_per_launch < 0 || P.sweeps_per_launch > 5 ||
        (P.sweeps_per_launch == 5 && !(P.ordering == CFD_ORDER_LEX && P.case_id == CFD_CAVITY)))
      throw Error(CFD_E_ARG, "sweeps_per_launch must be 0 (auto), 1, 2, 3, 4 or 5 (the cavity's lexicographic order)");
    if (P.sweeps_per_launch == 3 && P.case_id != CFD_CAVITY && P.ordering == CFD_ORDER_RB)
      throw Error(CFD_E_ARG, "three red-black sweeps per launch are implemented for the cavity only");
    if (P.sweeps_per_launch >= 1 && P.sweeps_per_launch != 4 && P.ordering == CFD_ORDER_LEX &&
        P.case_id != CFD_CAVITY && P.case_id != CFD_RAYLEIGH_BENARD)
      throw Error(CFD_E_ARG, "the open cases' lexicographic-order kernel runs 4 sweeps per launch (0: auto)");
    if (P.sweeps_per_launch == 4 && P.ordering == CFD_ORDER_RB && P.proof_test == CFD_OFF)
      throw Error(CFD_E_ARG, "four red-black sweeps per launch need the proof-mode test (proof_test != CFD_OFF)");
    for (int sw : {P.proof_test, P.small_solve, P.overlap})
      if (sw < CFD_AUTO || sw > CFD_OFF) throw Error(CFD_E_ARG, "proof_test / small_solve / overlap must be a cfd_switch");
    if (P.ordering != CFD_ORDER_RB && P.ordering != CFD_ORDER_LEX) throw Error(CFD_E_ARG, "unknown ordering");
    // (the cavity's lexicographic solve runs on the multi-block wavefront kernel
    // at any size; the open cases on the one-workgroup kernel)
    if (P.ordering == CFD_ORDER_LEX && P.case_id == CFD_BACKSTEP && !step_lexw_ok() && (P.nx + P.ny) / 3 + 8 >= LEX_WIN)
      throw Error(CFD_E_ARG, "lexicographic ordering of a backwards step with a block under 2 cells wide or high "
                             "supports nx + ny < 12000");
    // (that step runs the one-workgroup kernel, solve_lex: one strip; rejected
    // here rather than at the first solve)
    if (P.ordering == CFD_ORDER_LEX && P.case_id == CFD_BACKSTEP && !step_lexw_ok() && (nstrips > 1 || comm))
      throw Error(CFD_E_ARG, "lexicographic ordering of a backwards step with a block under 2 cells wide or high "
                             "runs on one strip (n_strips = 1, no ranks)");
#if CFD_WT_STORE
    // (write-through p_out stores address a strip's buffer with 32-bit buffer records)
    if ((double)(P.ny + 2 * HALO + 2) * (double)(((P.nx + 3) + 15) / 16 * 16) * 8.0 >= 4294967295.0)
      throw Error(CFD_E_ARG, "the CFD_WT_STORE build addresses p buffers below 4 GiB: grid too large");
#endif
    if (P.case_id == CFD_BACKSTEP && (P.step_i <= 0 || P.step_i >= P.nx))
      throw Error(CFD_E_ARG, "Step location is outside computational domain!");
    if (P.case_id == CFD_BACKSTEP && (P.inlet_jmax < 1 || P.inlet_jmax > P.ny))
      throw Error(CFD_E_ARG, "inlet height is outside computational domain");
  }

  bool multi() const { return S.size() > 1 || comm != nullptr; }

  // ------------------------------------------------------------ halos --
  // Copy `depth` owned boundary rows of buffer b into the neighbours' halos.
  void exchange(int b, int depth, hipStream_t xs = nullptr) {
    if (!xs) xs = st;
    if (S.size() > 1) {
      for (size_t k = 0; k + 1 < S.size(); ++k) {
        Strip& lo = S[k];
        Strip& up = S[k + 1];
        const size_t cnt = (size_t)depth * pitch * sizeof(double);
        const int ja = lo.g.j1 - depth + 1;  // lower strip's top rows -> upper's lower halo
        HIPC(hipMemcpyAsync(up.b[b] + (size_t)(ja - up.g.row_lo) * pitch, lo.b[b] + (size_t)(ja - lo.g.row_lo) * pitch,
                            cnt, hipMemcpyDeviceToDevice, xs));
        const int jb = up.g.j0;  // upper strip's bottom rows -> lower's upper halo
        HIPC(hipMemcpyAsync(lo.b[b] + (size_t)(jb - lo.g.row_lo) * pitch, up.b[b] + (size_t)(jb - up.g.row_lo) * pitch,
                            cnt, hipMemcpyDeviceToDevice, xs));
      }
    }
    if (comm && comm->nranks > 1) {
      Strip& s = S[0];
      const Geo& g = s.g;
      double* base = s.b[b];
      const size_t cnt = (size_t)depth * pitch;
      auto row = [&](int j) { return base + (size_t)(j - g.row_lo) * pitch; };
      comm_halo_exchange(comm, row(g.j0), row(g.j0 - depth), comm->rank > 0 ? comm->rank - 1 : -1,
                         row(g.j1 - depth + 1), row(g.j1 + 1), comm->rank < comm->nranks - 1 ? comm->rank + 1 : -1,
                         cnt, xs);
    }
  }

  // ------------------------------------------------------------- phases --
  void apply_bc(bool tentative) {
    const int bu = tentative ? B_US : B_U, bv = tentative ? B_VS : B_V;
    for (auto& s : S) {
      const Geo& g = s.g;
      const int n = std::max(P.nx + 1, g.wj1 - g.wj0 + 1);
      const dim3 grid((n + 255) / 256);
      if (P.case_id == CFD_CAVITY) {
        if (tentative) continue;  // the cavity never applies BCs to u*, v*
        bc_cavity_kernel<<<grid, 256, 0, st>>>(g, C, s.b[bu], s.b[bv]);
        check_launch("bc_cavity");
      } else {
        bc_open_kernel<<<grid, 256, 0, st>>>(g, C, s.b[bu], s.b[bv]);
        check_launch("bc_open");
        if (P.case_id == CFD_BACKSTEP) {
          const int box_i1 = std::min(P.step_i + 1, P.nx);
          const int box_j0 = std::max(P.inlet_jmax, g.wj0);
          const int box_j1 = std::min(P.ny, g.wj1);
          if (box_j1 >= box_j0) {
            const dim3 gf((box_i1 + 1 + 63) / 64, box_j1 - box_j0 + 1);
            bc_step_faces_kernel<<<gf, 64, 0, st>>>(g, C, s.b[bu], s.b[bv], box_i1, box_j0);
            check_launch("bc_step_faces");
          }
        }
      }
    }
  }

  void compute_tentative() {
    if (multi()) {
      exchange(B_U, 1);
      exchange(B_V, 1);
    }
    for (auto& s : S) {
      const int ct = P.nx / TENT_TWC + 1, rows = s.g.j1 - s.g.j0 + 1;
      const int th = std::max(1, std::min(tent_th, rows));  // rows per band (tuned: 64)
      const int tiles = ct * ((rows + th - 1) / th);
      tentative_kernel<<<(tiles + 3) / 4, 256, 0, st>>>(s.g, C, s.b[B_U], s.b[B_V], s.b[B_US], s.b[B_VS], th, ct);
      check_launch("tentative");
    }
  }

  // grid of the cavity's column-pair passes (cavity_source_kernel,
  // cavity_resmax_kernel): 128 columns x 4 owned interior rows per block
  dim3 pair_grid(const Strip& s) const {
    const int rows = std::min(s.g.j1, P.ny) - std::max(s.g.j0, 1) + 1;
    return dim3(P.nx / 128 + 1, std::max(1, (rows + 3) / 4));
  }

  bool srcmax_ready = false;  // srcmax holds max|f| of the current source (reduced by the source passes)

  void build_source() {
    HIPC(hipMemsetAsync(srcmax, 0, RES_SHARDS * SHARD_STRIDE * sizeof(double), st));
    if (multi()) exchange(B_VS, 1);
    for (auto& s : S) {
      if (P.case_id == CFD_CAVITY) {
        cavity_source_kernel<<<pair_grid(s), 256, 0, st>>>(s.g, C, s.b[B_US], s.b[B_VS], s.b[B_F], srcmax);
      } else {
        source_kernel<<<s.grid2d, 256, 0, st>>>(s.g, C, s.b[B_US], s.b[B_VS], s.b[B_F], partials + s.part_off, srcmax);
      }
      check_launch("source");
    }
    if (P.case_id != CFD_CAVITY) {
      if (P.ordering == CFD_ORDER_LEX && ranks()) {  // the same chain, rank to rank
        seq_sum_ranks(B_F, -1, 0, total);
      } else if (P.ordering == CFD_ORDER_LEX) {  // the reference's sequential sum, bit for bit (strips in order)
        for (size_t q = 0; q < S.size(); ++q)
          seq_sum(S[q], S[q].b[B_F], nullptr, 0, total, q > 0);
      } else {
        sum_partials_kernel<<<1, 256, 0, st>>>(partials, (int)npart, total);
      }
      check_launch("sum_partials");
      if (ranks() && P.ordering != CFD_ORDER_LEX) comm_allreduce_sum(comm, total, 1, st);
      for (auto& s : S) {
        subtract_mean_kernel<<<s.grid2d, 256, 0, st>>>(s.g, C, s.b[B_F], total, fluid_count, srcmax);
        check_launch("subtract_mean");
      }
    }
    srcmax_ready = true;
  }

  // Tolerance from the current source (computed inside the reference's solve).
  void solve_tolerance() {
    if (!srcmax_ready) {  // the source came from the host: reduce it here
      HIPC(hipMemsetAsync(srcmax, 0, RES_SHARDS * SHARD_STRIDE * sizeof(double), st));
      for (auto& s : S) {
        srcmax_kernel<<<s.grid2d, 256, 0, st>>>(s.g, C, s.b[B_F], srcmax);
        check_launch("srcmax");
      }
      srcmax_ready = true;
    }
    if (comm && comm->nranks > 1) comm_allreduce_max(comm, srcmax, RES_SHARDS * SHARD_STRIDE, st);
    tol_kernel<<<1, 64, 0, st>>>(C, srcmax, tolv);
    check_launch("tol");
  }

  // Sizing of the wave-march kernels: column tiles of `twc` output columns,
  // each split into bands so that one resident round covers the strip.
  void wave_bands(int rows, int twc, int resident, int& ctiles, int& th, int& nbands) const {
    ctiles = (P.nx + 2 + twc - 1) / twc;
    const int per_tile = std::max(1, resident / (ctiles * (int)S.size()));
    const int bands = std::max(1, std::min(per_tile, (rows + march_min_th - 1) / march_min_th));
    th = (rows + bands - 1) / bands;
    nbands = (rows + th - 1) / th;
  }

  // Rows one interior wave marches beyond its band (both sides together, plus
  // the parity alignment row) for an n-sweep launch: the cavity's pipeline has
  // depth 2n+1, the open cases' pair pipeline 7.
  // an n-sweep launch that runs open.hip's proof march (its plans may carry the step's left class)
  bool open_proof_n(int n) const { return P.case_id != CFD_CAVITY && n >= 3 && proof_launch; }

  int march_extra(int n) const { return (P.case_id == CFD_CAVITY || n == 4) ? 2 * (2 * n + 1) + 1 : 15; }

  // Tiling of an n-sweep launch over rows [lo0, hi0) + [lo1, hi1) with at most
  // `waves` waves (one resident round). Interior column tiles: bands of th
  // rows, marched in groups of 10 over th + march_extra rows, so th + extra is
  // a multiple of 10. The two boundary column tiles march slower (masks):
  // shorter bands, pair_edge_pct % of the interior march.
  // left_class (the step's proof launches, open.hip): the column tiles over
  // the step's block (left of its column and across it) become their own
  // class (PairPlan::nl / ncx): interior-path bands below the block, short
  // masked bands next to its lower edge and above it.
  PairPlan multi_plan(int lo0, int hi0, int lo1, int hi1, int waves, int n, int max_th = 1 << 30,
                      int edge_pct = -1, int twc = PAIR_TWC, int ex = -1, bool left_class = false) const {
    if (edge_pct < 0) edge_pct = pair_edge_pct;
    PairPlan pl{};
    pl.ctiles = (P.nx + 2 + twc - 1) / twc;
    pl.lo0 = lo0; pl.hi0 = hi0; pl.lo1 = lo1; pl.hi1 = hi1;
    if (P.case_id == CFD_BACKSTEP) {
      // interior column tiles across the step's column (neither left of it,
      // kernels.hpp: c0 + 128 <= step_i - 1, nor right, c0 > step_i + 1) march
      // with per-cell masks: band them like the boundary tiles
      int nx_found = 0;
      for (int ct = 1; ct + 1 < pl.ctiles && nx_found < 2; ++ct) {
        const int c0 = ct * PAIR_TWC - 8;
        if (!(c0 > C.step_i + 1) && !(c0 + 128 <= C.step_i - 1)) {
          (nx_found == 0 ? pl.cxa : pl.cxb) = ct + 1;
          ++nx_found;
        }
      }
    }
    const int rows = (hi0 - lo0) + (hi1 - lo1);
    const int rmax = std::max(hi0 - lo0, hi1 - lo1);
    if (ex < 0) ex = march_extra(n);
    auto nbands = [](int lo, int hi, int t) { return hi > lo ? (hi - lo + t - 1) / t : 0; };
    // the block's column class (PairPlan::nl / ncx): column tiles 1 .. cxa-2
    // (wholly left of the step's column) and the crossing ones; rows [lo0, lz)
    // interior-column bands (every row the march reads below the block's
    // lower edge row: open.hip cols_in), [lz, le) short masked bands, above
    // that the top ghost row (left tiles) or every row (crossing tiles)
    const int cx_last = pl.cxb > 0 ? pl.cxb - 1 : pl.cxa - 1;  // the last crossing tile
    const bool lc = left_class && P.case_id == CFD_BACKSTEP && pl.cxa > 1 && cx_last < pl.ctiles - 1 && hi1 <= lo1;
    if (lc) {
      pl.nl = pl.cxa - 2;
      pl.ncx = pl.cxb > 0 ? 2 : 1;
      pl.cxa = pl.cxb = 0;  // (the crossing tiles leave the boundary class)
      pl.lz = std::max(lo0, std::min(hi0, C.inlet_jmax - (2 * n + 2)));
      pl.le = std::max(pl.lz, std::min(hi0, C.inlet_jmax + 2));
      pl.lt = hi0;  // (ghost row ny + 1 in the range: set with `the` below)
    }
    auto left_bands = [&] {
      if (!lc) return;
      pl.nlf = nbands(lo0, pl.lz, pl.th);
      pl.nle = nbands(pl.lz, pl.le, pl.the);
      if (hi0 == P.ny + 2) pl.lt = std::max(pl.le, hi0 - pl.the);
      pl.nlt = nbands(pl.lt, hi0, pl.the);
      pl.nxt = nbands(pl.le, hi0, pl.the);
    };
    int nb = std::max(1, std::min(waves / std::max(1, pl.ctiles), (rows + march_min_th - 1) / march_min_th));
    nb = std::max(nb, (rows + max_th - 1) / max_th);
    for (;; --nb) {  // most interior bands whose tiles (boundary tiles included) fit one round
      pl.th = std::max(1, std::min(rmax, ((rows + nb - 1) / nb + ex + 9) / 10 * 10 - ex));
      if (pl.th > max_th) {  // (lexw: one wave marches at most max_th rows)
        pl.th = max_th;
        pl.the = std::max(8, std::min(rmax, (pl.th + ex) * edge_pct / 100 - ex));
        pl.nb0 = nbands(lo0, hi0, pl.th);
        pl.nb1 = nbands(lo1, hi1, pl.th);
        pl.nbe0 = nbands(lo0, hi0, pl.the);
        pl.nbe1 = nbands(lo1, hi1, pl.the);
        left_bands();
        break;
      }
      pl.the = std::max(8, std::min(rmax, (pl.th + ex) * edge_pct / 100 - ex));
      pl.nb0 = nbands(lo0, hi0, pl.th);
      pl.nb1 = nbands(lo1, hi1, pl.th);
      pl.nbe0 = nbands(lo0, hi0, pl.the);
      pl.nbe1 = nbands(lo1, hi1, pl.the);
      left_bands();
      if (plan_waves(pl) <= waves || nb == 1) break;
    }
    return pl;
  }

  // One launch of poisson_multi_kernel: iterations k .. k+n-1 (n = 2, or 3 for
  // the cavity), testing iterations [ka, kb] first (empty: ka > kb).
  template <int CASE>
  void launch_multi(int n, const PairPlan& pl, const Geo& g, const double* pin, double* pout, const double* f,
                    const PoissonCtl& ctl, int k, int ka, int kb, hipStream_t stream, bool replay = false) {
    // bit 2: no test at all (the solve has already stopped); bit 7: the tested
    // window holds proof ratios (it was computed by a proof-mode launch)
    const int fl = march_flags | (replay ? 4 : 0) | (window_proof ? 128 : 0);
    const int ntiles = plan_waves(pl);
    if (ntiles == 0) return;
    const dim3 grid((ntiles + 3) / 4);
    if constexpr (CASE == CAVITY) {
      if (n == 4) {  // proof mode only (Solver::proof_ns)
        if (!proof_launch || replay) throw Error(CFD_E_STATE, "four sweeps per launch: proof mode only");
        poisson_multi_kernel<CASE, 4, true><<<grid, 256, 0, stream>>>(g, C, pin, pout, f, ctl, k, ka, kb, pl, fl);
        return;
      }
      if (n == 3) {
        if (proof_launch && !replay)
          poisson_multi_kernel<CASE, 3, true><<<grid, 256, 0, stream>>>(g, C, pin, pout, f, ctl, k, ka, kb, pl, fl);
        else
          poisson_multi_kernel<CASE, 3><<<grid, 256, 0, stream>>>(g, C, pin, pout, f, ctl, k, ka, kb, pl, fl);
        return;
      }
    }
    if constexpr (CASE != CAVITY) {
      if (n >= 3) {  // proof mode only (open.hip)
        if (!proof_launch || replay) throw Error(CFD_E_STATE, "three or four sweeps per launch: proof mode only");
        open_proof_launch(CASE, n, g, C, pin, pout, f, ctl, k, ka, kb, pl, fl, stream);
        return;
      }
    }
    poisson_multi_kernel<CASE, 2><<<grid, 256, 0, stream>>>(g, C, pin, pout, f, ctl, k, ka, kb, pl, fl);
  }

  // One SOR launch over every strip: iterations k .. k+n-1, testing [ka, kb].
  template <int CASE>
  void launch_poisson(const double* const* pin, double* const* pout, int k, int n, int ka, int kb, bool replay) {
    PoissonCtl ctl{ring, tolv, stop, P.check_every};
    if (tile_on) {  // one strip (plan_tiles)
      tile_launch(P.case_id, proof_launch && !replay, S[0].g, C, pin[0], pout[0], S[0].b[B_F], ctl, k, ka, kb, n,
                  tplan, march_flags | (replay ? 4 : 0) | (window_proof ? 128 : 0), st);
      check_launch("poisson (tile)");
      return;
    }
    for (size_t q = 0; q < S.size(); ++q) {
      const Geo& g = S[q].g;
      const int rows = g.wj1 - g.wj0 + 1;
      int ctiles, th, nbands;
      if (n >= 2) {
        const PairPlan pl = multi_plan(g.wj0, g.wj1 + 1, 0, 0, resident_pair_waves / (int)S.size(), n, 1 << 30, -1,
                                       PAIR_TWC, -1, open_proof_n(n));
        launch_multi<CASE>(n, pl, g, pin[q], pout[q], S[q].b[B_F], ctl, k, ka, kb, st, replay);
      } else {
        wave_bands(rows, 128 - 8, resident_waves, ctiles, th, nbands);
        const int nblk = (ctiles * nbands + 3) / 4;
        poisson_wave_kernel<CASE><<<nblk, 256, 0, st>>>(g, C, pin[q], pout[q], S[q].b[B_F], ctl, k, ka, kb, th, ctiles,
                                                         nbands, march_flags | (replay ? 4 : 0) | (window_proof ? 128 : 0));
      }
    }
    check_launch("poisson");
  }

  // st waits for everything enqueued on st_b so far
  void join_b() {
    if (b_pending) {
      HIPC(hipStreamWaitEvent(st, ev_bnd[last_bnd], 0));
      b_pending = false;
    }
  }

  // all-reduce (max) of the residual slots of iterations k .. k+n-1 that are tested
  // (slots adjacent in the ring go in one call: one RCCL latency per launch)
  void allreduce_slots(int k, int n, hipStream_t xs) {
    constexpr size_t SLOT = (size_t)RES_SHARDS * SHARD_STRIDE;
    int run0 = -1, runn = 0;  // ring slots [run0, run0 + runn) pending
    auto flush = [&] {
      if (runn > 0) comm_allreduce_max(comm, ring + (size_t)run0 * SLOT, SLOT * runn, xs);
      runn = 0;
    };
    for (int kk = k; kk < k + n && kk <= P.max_iters; ++kk) {
      if (!(kk % P.check_every == 0 || kk == P.max_iters)) continue;
      const int sl = kk & (RING - 1);
      if (runn > 0 && sl == run0 + runn) {
        ++runn;
      } else {
        flush();
        run0 = sl;
        runn = 1;
      }
    }
    flush();
  }

  // Launch m (n >= 2 sweeps) on a rank with halo overlap. st_b: exchange of
  // the launch's input rows, the all-reduce of launch m-1's residuals (tested
  // by launch m+1: lagged), then the rows within OVL_ROWS of each neighbour
  // (their cone reaches the interior rows of launch m-1: wait for it). st: the
  // interior rows (they never read halo rows; wait for launch m-1's boundary
  // rows), concurrently.
  template <int CASE>
  void multi_overlapped(int m, int k, int n, int ka, int kb, int bin, int bout) {
    const Strip& s = S[0];
    double* pin = s.b[bin];
    double* pout = s.b[bout];
    const Geo& g = s.g;
    const int lo_b = comm->rank > 0 ? OVL_ROWS : 0;
    const int hi_b = comm->rank < comm->nranks - 1 ? OVL_ROWS : 0;
    const int e = m & 1, pe = e ^ 1;
    PoissonCtl ctl{ring, tolv, stop, P.check_every};
    if (m == 0) {  // st_b starts after st's work so far (source, tolerance, f halos)
      HIPC(hipEventRecord(ev_sync, st));
      HIPC(hipStreamWaitEvent(st_b, ev_sync, 0));
    }
    exchange(bin, HALO, st_b);
    if (m > 0) {
      HIPC(hipStreamWaitEvent(st_b, ev_int[pe], 0));
      flush_allreduce(st_b);  // launch m-1's residuals, tested by launch m+1
    }
    PairPlan pb{};
    pb.ctiles = (P.nx + 2 + PAIR_TWC - 1) / PAIR_TWC;
    pb.th = pb.the = OVL_ROWS;
    pb.lo0 = g.wj0; pb.hi0 = g.wj0 + lo_b;
    pb.lo1 = g.wj1 + 1 - hi_b; pb.hi1 = g.wj1 + 1;
    pb.nb0 = pb.nbe0 = lo_b ? 1 : 0;
    pb.nb1 = pb.nbe1 = hi_b ? 1 : 0;
    launch_multi<CASE>(n, pb, g, pin, pout, s.b[B_F], ctl, k, ka, kb, st_b);
    if (m > 0) HIPC(hipStreamWaitEvent(st, ev_bnd[pe], 0));
    const PairPlan pi = multi_plan(g.wj0 + lo_b, g.wj1 + 1 - hi_b, 0, 0, resident_pair_waves - 2 * pb.ctiles, n,
                                   1 << 30, -1, PAIR_TWC, -1, open_proof_n(n));
    launch_multi<CASE>(n, pi, g, pin, pout, s.b[B_F], ctl, k, ka, kb, st);
    check_launch("poisson (overlapped)");
    HIPC(hipEventRecord(ev_int[e], st));
    HIPC(hipEventRecord(ev_bnd[e], st_b));
    ar_pending = {k, n, proof_launch};
    last_bnd = e;
    b_pending = true;
    ++n_overlapped;
  }

  // SOR launch number m (0-based) of a solve starting in buffer `base`: reads
  // buffer (base+m) mod nbufs, writes the next. Iterations k .. k+n-1; tests
  // iterations [ka, kb] first. replay: recomputes iterations of a launch that
  // already ran (no test, no all-reduce).
  void poisson_launch(int m, int k, int n, int base, int ka, int kb, bool replay) {
    const int bin = pbuf((base + m) % nbufs());
    const int bout = pbuf((base + m + 1) % nbufs());
    if (overlap && n >= 2 && !replay) {
      if (P.case_id == CFD_CAVITY) multi_overlapped<CAVITY>(m, k, n, ka, kb, bin, bout);
      else if (P.case_id == CFD_CHANNEL) multi_overlapped<CHANNEL>(m, k, n, ka, kb, bin, bout);
      else multi_overlapped<BACKSTEP>(m, k, n, ka, kb, bin, bout);
      return;
    }
    join_b();
    flush_allreduce(st);  // an overlapped launch before this one
    if (multi()) exchange(bin, n >= 2 ? HALO : 4);
    std::vector<const double*> pin(S.size());
    std::vector<double*> pout(S.size());
    for (size_t q = 0; q < S.size(); ++q) {
      pin[q] = S[q].b[bin];
      pout[q] = S[q].b[bout];
    }
    if (P.case_id == CFD_CAVITY) launch_poisson<CAVITY>(pin.data(), pout.data(), k, n, ka, kb, replay);
    else if (P.case_id == CFD_CHANNEL) launch_poisson<CHANNEL>(pin.data(), pout.data(), k, n, ka, kb, replay);
    else launch_poisson<BACKSTEP>(pin.data(), pout.data(), k, n, ka, kb, replay);
    if (comm && comm->nranks > 1 && !replay) allreduce_slots(k, n, st);
  }

  // solverPressurePoisson (cavity-01.cpp:609-690, channel-01.cpp:635-688,
  // backwards_step-01.cpp:872-939). Requires build_source() first.
  // Reference-order SOR (poisson_lex_kernel): one persistent workgroup.
  void solve_lex(cfd_step_info* out) {
    if (S.size() != 1 || comm) throw Error(CFD_E_STATE, "lexicographic ordering needs a single-strip solver");
    Strip& s = S[0];
    const int base = pcur;
    const size_t bytes = (size_t)s.g.nrows * pitch * sizeof(double);
    double* X0 = s.b[pbuf(base)];       // (lex: single strip, no ranks -> two buffers)
    double* X1 = s.b[pbuf(base ^ 1)];
    if (P.case_id == CFD_CAVITY) {  // cavity-01.cpp:610-611: zero field, zero ghosts
      HIPC(hipMemsetAsync(X0, 0, bytes, st));
      HIPC(hipMemsetAsync(X1, 0, bytes, st));
    }
    solve_tolerance();
    HIPC(hipMemcpyAsync(s.b[B_PL], X0, bytes, hipMemcpyDeviceToDevice, st));
    int* d_it = stop;
    double* d_res = total + 2;
    HIPC(hipEventRecord(ev_a, st));
    if (P.case_id == CFD_CAVITY)
      poisson_lex_kernel<CAVITY><<<1, 1024, 0, st>>>(s.g, C, X0, X1, s.b[B_PL], s.b[B_F], tolv, P.max_iters, d_it, d_res);
    else if (P.case_id == CFD_CHANNEL)
      poisson_lex_kernel<CHANNEL><<<1, 1024, 0, st>>>(s.g, C, X0, X1, s.b[B_PL], s.b[B_F], tolv, P.max_iters, d_it, d_res);
    else
      poisson_lex_kernel<BACKSTEP><<<1, 1024, 0, st>>>(s.g, C, X0, X1, s.b[B_PL], s.b[B_F], tolv, P.max_iters, d_it, d_res);
    check_launch("poisson_lex");
    HIPC(hipEventRecord(ev_b, st));
    int iters = 0;
    double res = 0;
    HIPC(hipMemcpyAsync(&iters, d_it, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(&res, d_res, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
    T.poisson_ms += ms;
    T.poisson_launches += 1;
    T.poisson_cell_updates += (long long)P.nx * P.ny * iters;
    pcur = (base + iters) & 1;
    if (out) {
      out->sor_iterations = iters;
      out->residual = res;
    }
  }

  // ---- lexicographic order, multi-block (lexw.hpp) ----
  int lexw_offset() const { return (P.nx + P.ny) / 2 + 192; }
  static int floordiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }
  // iterations whose residual every cell has contributed after launch m (H0 = 2 + 2NS m)
  int lexw_done(int m, int ns) const { return m < 0 ? 0 : floordiv(2 + 2 * ns * m + 2 * ns - 2 - P.nx - P.ny, 2) + 1; }

  // steady: every cell active in every half-sweep of the launch and in the
  // previous launch's last one (no activity masks: the leaner kernel)
  // backwards step, reference order: the block's ghost constants set before
  // the march (lexw.hpp step_presolid_kernel), so that the column tiles left
  // of the step's column end at the block's bottom row and march as a channel
  // below it (flags bit 3; CFD_TUNE_LEXW_LEFT 0: the per-cell masked march)
#ifndef CFD_LEXW_XSPLIT
#define CFD_LEXW_XSPLIT 3
#endif
  // the step's interior column tiles that cross its column (the per-cell solid
  // rules at the block's edge): xa .. xa + xn - 1, xa = -1 if none
  void lexw_cross_tiles(int ns, const PairPlan& pl, int* xa, int* xn) const {
    const int twc = lexw_twc(ns), ch = lexw_ch(ns), si = C.step_i;
    *xa = -1;
    *xn = 0;
    for (int ct = 1; ct + 1 < pl.ctiles; ++ct) {
      const int c0 = ct * twc - ch;
      const bool left = c0 + 127 <= si - 1 && lexw_left_class();
      if (!left && c0 <= si + 1) {
        if (*xa < 0) *xa = ct;
        *xn = ct - *xa + 1;
      }
    }
  }
  bool lexw_left_class() const { return P.case_id == CFD_BACKSTEP && lexw_left; }
  void lexw_presolid() {
    if (!lexw_left_class()) return;
    for (auto& s : S)
      for (int b : {0, 1}) {
        const int n = std::max(C.step_i, P.ny) + 1;
        step_presolid_kernel<<<(n + 255) / 256, 256, 0, st>>>(s.g, C, s.b[pbuf(b)]);
        check_launch("step_presolid");
      }
  }

  void launch_lexw(int ns, bool steady, bool sample, const PairPlan& pl, const Geo& g, const double* pin,
                   double* pout, const double* f, const LexCtl& L, int H0, int K, int ka, int kb, bool replay,
                   int waves) {
    const int fl = (replay ? 4 : 0) | (lexw_left_class() ? 8 : 0) | (lexw_updown ? 16 : 0);
    const int ne = pl.ctiles >= 2 ? 2 : 1;
    int ntiles = ne * (pl.nbe0 + pl.nbe1) + (pl.ctiles - ne) * (pl.nb0 + pl.nb1);
    LexRamp rp{};
    if (!steady) {
      // ramp launch: tile only the rows it touches (lexw_rows), bands of the
      // shortest height whose tiles fit one resident round, at most the
      // steady plan's (at that every ramp launch fits: it touches fewer rows)
      int rl = 1 << 30, rh = -1;
      long long tot = 0;
      std::vector<std::pair<int, int>> rr(pl.ctiles);
      for (int c = 0; c < pl.ctiles; ++c) {
        lexw_rows(g, H0, K, ns, c, &rr[c].first, &rr[c].second, P.case_id != CFD_CAVITY);
        if (rr[c].second >= rr[c].first) {
          rl = std::min(rl, rr[c].first);
          rh = std::max(rh, rr[c].second);
          tot += rr[c].second - rr[c].first + 1;
        }
      }
      if (rh < rl) return;
      const int ex = lexw_extra(ns);
      rp.wsplit = CFD_LEXW_WALL_SPLIT;
      if (P.case_id == CFD_BACKSTEP && CFD_LEXW_XSPLIT > 1) {  // the step's crossing tiles (as the steady split)
        int xa, xn;
        lexw_cross_tiles(ns, pl, &xa, &xn);
        if (xa >= 0) {
          rp.xa = xa;
          rp.xn = xn;
          rp.xreach = 4 * ns + 4 - (C.inlet_jmax + 1);
        }
      }
      auto build = [&](int th) {  // fills rp for band height th; returns the tile count
        rp.th = th;
        rp.row0 = rl;
        rp.nb = (rh - rl) / th + 1;
        int n = 0;
        for (int b = 0; b < rp.nb; ++b) {
          const int blo = rl + b * th, bhi = blo + th - 1;
          int ca = -1, cb = -2;
          for (int c = 0; c < pl.ctiles; ++c)
            if (std::max(blo, rr[c].first) <= std::min(bhi, rr[c].second)) {
              if (ca < 0) ca = c;
              cb = c;
            }
          if (ca < 0) ca = 0, cb = -1;  // (an empty band: no tiles)
          rp.band[b] = ((unsigned)n << 16) | ((unsigned)ca << 8) | (unsigned)(cb < 0 ? 0 : cb);
          if (cb < 0) rp.band[b] = ((unsigned)n << 16) | 1u << 8;  // ca 1 > cb 0: empty
          n += std::max(0, cb - ca + 1);
          if (cb >= ca) {  // a second wave per split tile (lexw.hpp lexw_ramp_waves: half bands)
            int ct, hf;
            n += lexw_ramp_waves(rp, pl.ctiles, b, ca, cb, 0, &ct, &hf);
          }
        }
        return n;
      };
      int th = (int)std::max<long long>(1, (tot + waves - 1) / std::max(1, waves));
      // (a floor on the band height trades idle wave slots for less pipeline fill per output row)
      th = std::max(th, pl.th * lexw_ramp_pct / 100);
      th = std::max(1, (th + ex + 9) / 10 * 10 - ex);
      while ((rh - rl) / th + 1 > LEXW_RAMP_BANDS) th += 10;
      ntiles = build(th);
      while (th < pl.th && ntiles > waves) ntiles = build(th += 10);
      if (th > pl.th) ntiles = build(th = std::max(pl.th, (rh - rl) / LEXW_RAMP_BANDS + 1));
      if (pl.ctiles > 255 || ntiles >= 65536) throw Error(CFD_E_ARG, "lexicographic ordering: grid too wide");
    }
    // the step's steady launches: the crossing column tiles' bands that reach
    // the block's edge as CFD_LEXW_XSPLIT shorter bands (lexw.hpp; they set
    // the launch's time: profiles/r5/step_8192x512_lex_stamps.json)
    PairPlan plx = pl;
    if (steady && P.case_id == CFD_BACKSTEP && CFD_LEXW_XSPLIT > 1 && pl.nb1 == 0 && pl.ctiles >= 3) {
      const int jb = C.inlet_jmax + 1;
      int xa, xn;
      lexw_cross_tiles(ns, pl, &xa, &xn);
      int xb = -1;
      for (int b = 0; b < pl.nb0 && xb < 0; ++b)
        if (std::min(pl.lo0 + (b + 1) * pl.th, pl.hi0) + 4 * ns + 4 >= jb) xb = b;
      if (xa >= 0 && xb >= 0) {
        plx.xa = xa;
        plx.xn = xn;
        plx.xb = xb;
        plx.xbn = pl.nb0 - xb;
        plx.xparts = CFD_LEXW_XSPLIT;
        ntiles += plx.xn * plx.xbn * (plx.xparts - 1);
      }
    }
    if (ntiles == 0) return;
    const dim3 grid((ntiles + 3) / 4);
#define CFD_LEXW_LAUNCH(CASE, NS, R, SM) \
  poisson_lexw_kernel<CASE, NS, R, SM><<<grid, 256, 0, st>>>(g, C, pin, pout, f, L, H0, K, ka, kb, plx, fl, rp)
    // (sampled residual rows: the 3-sweep kernels, the default; 1 and 2 sweeps evaluate every row)
    if (P.case_id == CFD_BACKSTEP && ns == 3) {  // (strips)
      if (sample) { if (steady) CFD_LEXW_LAUNCH(BACKSTEP, 3, false, true); else CFD_LEXW_LAUNCH(BACKSTEP, 3, true, true); }
      else { if (steady) CFD_LEXW_LAUNCH(BACKSTEP, 3, false, false); else CFD_LEXW_LAUNCH(BACKSTEP, 3, true, false); }
    } else if (P.case_id == CFD_BACKSTEP) {
      if (sample) { if (steady) CFD_LEXW_LAUNCH(BACKSTEP, 4, false, true); else CFD_LEXW_LAUNCH(BACKSTEP, 4, true, true); }
      else { if (steady) CFD_LEXW_LAUNCH(BACKSTEP, 4, false, false); else CFD_LEXW_LAUNCH(BACKSTEP, 4, true, false); }
    } else if (P.case_id == CFD_CHANNEL && ns == 3) {  // (strips)
      if (sample) { if (steady) CFD_LEXW_LAUNCH(CHANNEL, 3, false, true); else CFD_LEXW_LAUNCH(CHANNEL, 3, true, true); }
      else { if (steady) CFD_LEXW_LAUNCH(CHANNEL, 3, false, false); else CFD_LEXW_LAUNCH(CHANNEL, 3, true, false); }
    } else if (P.case_id == CFD_CHANNEL) {
      if (sample) { if (steady) CFD_LEXW_LAUNCH(CHANNEL, 4, false, true); else CFD_LEXW_LAUNCH(CHANNEL, 4, true, true); }
      else { if (steady) CFD_LEXW_LAUNCH(CHANNEL, 4, false, false); else CFD_LEXW_LAUNCH(CHANNEL, 4, true, false); }
    } else if (ns == 5) {
      if (sample) { if (steady) CFD_LEXW_LAUNCH(CAVITY, 5, false, true); else CFD_LEXW_LAUNCH(CAVITY, 5, true, true); }
      else { if (steady) CFD_LEXW_LAUNCH(CAVITY, 5, false, false); else CFD_LEXW_LAUNCH(CAVITY, 5, true, false); }
    } else if (ns == 4) {
      if (sample) { if (steady) CFD_LEXW_LAUNCH(CAVITY, 4, false, true); else CFD_LEXW_LAUNCH(CAVITY, 4, true, true); }
      else { if (steady) CFD_LEXW_LAUNCH(CAVITY, 4, false, false); else CFD_LEXW_LAUNCH(CAVITY, 4, true, false); }
    } else if (ns == 1) { if (steady) CFD_LEXW_LAUNCH(CAVITY, 1, false, false); else CFD_LEXW_LAUNCH(CAVITY, 1, true, false); }
    else if (ns == 2) { if (steady) CFD_LEXW_LAUNCH(CAVITY, 2, false, false); else CFD_LEXW_LAUNCH(CAVITY, 2, true, false); }
    else if (sample) { if (steady) CFD_LEXW_LAUNCH(CAVITY, 3, false, true); else CFD_LEXW_LAUNCH(CAVITY, 3, true, true); }
    else { if (steady) CFD_LEXW_LAUNCH(CAVITY, 3, false, false); else CFD_LEXW_LAUNCH(CAVITY, 3, true, false); }
#undef CFD_LEXW_LAUNCH
  }

  // K lexicographic iterations of every cell as launches m = 0.. (half-sweeps
  // H0 = 2 + 2NS m ..), starting from buffer `base`; with tests, launch m first
  // tests the iterations completed by launch m-1, from iteration ka0 (0: the
  // primed initial residual). Iterations >= kexact are evaluated on every cell
  // (full launches from the first one that evaluates iteration kexact
  // anywhere); below it on sampled rows (3-sweep kernel). Returns the launches
  // run (the result is in pbuf((base + launches) % 2)); *code = 0 (no stop
  // before K), 1 (the reference stops at *kstop) or 2 (*kstop left open: no
  // sampled cell exceeds the tolerance).
  int run_lexw(int base, int K, bool tests, int kexact, int ka0, int* kstop, int* code, bool time_steady) {
    const int ns = lexw_ns();
    // the last half-sweep: cell (ny, nx)'s K-th update, and for the open cases
    // the top ghost (ny+1, nx)'s K-th copy one half-sweep later (lxo_row)
    const int Hlast = P.nx + P.ny + 2 * (K - 1) + (P.case_id != CFD_CAVITY ? 1 : 0);
    const int nl = (Hlast - 2) / (2 * ns) + 1;  // last launch covers Hlast
    const int kmax = lexw_offset();
    LexCtl L{lexbits, (int)(lexbits_words / LEXW_SHARDS), kmax, tolv, stop, kexact, cscr};
    // the residual of iteration k of cell (j,i) (half-sweep i+j+2(k-1)) is
    // evaluated in the launch holding half-sweep i+j+2k-1; the corner cell's
    // (i+j = 2) is the first: launches from m_full evaluate iterations >=
    // kexact everywhere. Replays (no tests) use the sampled kernel throughout.
    // (kexact >= K: no iteration the solve tests is evaluated everywhere)
    const int m_full = (!tests || kexact >= K) ? INT32_MAX : (ns >= 3) ? (2 * kexact - 1) / (2 * ns) : 0;
    std::vector<PairPlan> plans(S.size());
    for (size_t q = 0; q < S.size(); ++q)
      plans[q] = multi_plan(S[q].g.wj0, S[q].g.wj1 + 1, 0, 0, resident_lexw_waves / (int)S.size(), ns,
                            ns >= 5 ? 90 : 96,  // (a wave's march steps + 9 <= 127: its iterations fit one 64-bit mask)
                            lexw_edge_pct, lexw_twc(ns), lexw_extra(ns));
    // steady launches of strip q: every cell the strip's launch touches (its
    // rows and the HALO rows on each side: i + j in [smin, smax]) active in
    // every half-sweep of the launch and of the previous one's last
    // (smax + 1 <= H0 <= smin + 2K - 2NS - 1, H0 = 2 + 2NS m; one strip:
    // smin = 2, smax = nx + ny). A strip of a tall grid (ranks) runs its own
    // steady window instead of the whole grid's, which starts only once the
    // last row has started.
    std::vector<int> qs0(S.size()), qs1(S.size());
    int ms0 = 0, ms1 = INT32_MAX;  // launches steady on every strip (timed)
    for (size_t q = 0; q < S.size(); ++q) {
      const Geo& g = S[q].g;
      const int smax = P.nx + std::min(P.ny, g.j1 + HALO), smin = 1 + std::max(1, g.j0 - HALO);
      qs0[q] = (smax - 1 + 2 * ns - 1) / (2 * ns);
      qs1[q] = floordiv(smin + 2 * K - 2 * ns - 3, 2 * ns);
      ms0 = std::max(ms0, qs0[q]);
      ms1 = std::min(ms1, qs1[q]);
    }
    const bool steady = time_steady && ms1 >= ms0;
    const int chunk = P.chunk > 0 ? P.chunk : 32;
    if (K >= 1) lexw_presolid();  // (both buffers hold the solve's input here)
    int tested = tests ? ka0 - 1 : K;  // highest iteration tested
    int reduced = tested;              // ranks: highest iteration whose bits are OR-ed over the ranks
    bool stopped = false;
    int m = 0, c = 0;
    *kstop = -1;
    *code = 0;
    while (m < nl && !stopped) {
      for (int jj = 0; jj < chunk && m < nl; ++jj, ++m) {
        int ka = 1, kb = 0;
        if (tests) {
          if (m == 0) {
            if (ka0 == 0) ka = kb = 0;
          } else {
            ka = tested + 1;
            kb = std::min(lexw_done(m - 1, ns), K - 1);
            if (ranks()) {  // (only bits OR-ed over the ranks are tested)
              if (m % LEXW_RED_EVERY == 0 && kb > reduced) {
                lexw_reduce_bits(L, reduced + 1, kb);
                reduced = kb;
              }
              kb = std::min(kb, reduced);
            }
          }
          if (ka <= kb) tested = kb;
        }
        const int bin = pbuf((base + m) % 2), bout = pbuf((base + m + 1) % 2);
        if (multi()) exchange(bin, HALO);
        if (steady && m == ms0) HIPC(hipEventRecord(ev_f0, st));
        for (size_t q = 0; q < S.size(); ++q)
          launch_lexw(ns, m >= qs0[q] && m <= qs1[q], m < m_full, plans[q], S[q].g, S[q].b[bin], S[q].b[bout],
                      S[q].b[B_F], L, 2 + 2 * ns * m, K, ka, kb, !tests, resident_lexw_waves / (int)S.size());
        check_launch("poisson_lexw");
        if (steady && m == ms1) HIPC(hipEventRecord(ev_f1, st));
      }
      if (tests) {
        HIPC(hipMemcpyAsync(h_stat + 2 * (c & 1), stop, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
        HIPC(hipEventRecord(ev_poll[c & 1], st));
        if (c > 0) {
          HIPC(hipEventSynchronize(ev_poll[(c - 1) & 1]));
          if (h_stat[2 * ((c - 1) & 1)] != 0) stopped = true;
        }
        ++c;
      }
    }
    if (tests) {
      HIPC(hipStreamSynchronize(st));
      HIPC(hipMemcpy(h_stat, stop, 2 * sizeof(int), hipMemcpyDeviceToHost));
      if (h_stat[0]) {
        *kstop = h_stat[1];
        *code = h_stat[0];
      } else if (tested < K - 1) {  // iterations completed by the last launches: tested here, in order
        if (ranks() && reduced < K - 1) {
          lexw_reduce_bits(L, std::max(reduced + 1, 1), K - 1);
          HIPC(hipStreamSynchronize(st));
        }
        std::vector<unsigned long long> hb(lexbits_words);
        HIPC(hipMemcpy(hb.data(), lexbits, lexbits_words * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        const size_t wps = lexbits_words / LEXW_SHARDS;
        for (int k = std::max(tested + 1, 1); k <= K - 1; ++k) {
          const int qb = kmax + k;
          unsigned long long w = 0;
          for (int sh = 0; sh < LEXW_SHARDS; ++sh) w |= hb[(size_t)sh * wps + (qb >> 6)];
          if (!((w >> (qb & 63)) & 1ull)) {
            *kstop = k;
            *code = (k >= kexact) ? 1 : 2;
            break;
          }
        }
      }
    }
    if (steady && m > ms1) {  // (both events recorded: the solve did not stop before the last steady launch)
      HIPC(hipEventSynchronize(ev_f1));
      float ms = 0.f;
      HIPC(hipEventElapsedTime(&ms, ev_f0, ev_f1));
      T.poisson_steady_ms += ms;
      T.poisson_steady_launches += ms1 - ms0 + 1;
    }
    return m;
  }

  // solverPressurePoisson in the reference's own sweep order, any grid size.
  //
  // The 3-sweep launches evaluate residuals on sampled rows (lexw.hpp
  // LX_SAMPLE): enough to prove that the loop goes on, far from convergence.
  // Iterations >= kexact are evaluated on every cell: from 64 before the
  // previous solve's stop when it converged, none when it was capped (the
  // bench). An iteration whose sampled rows all meet the tolerance is left
  // open (code 2): the field after it is rebuilt (replay) and its exact
  // max-norm residual decides; if the loop goes on, the solve continues from
  // that field with every cell evaluated (the lexicographic sweep depends on
  // nothing but the current field, so iteration q of the continuation is the
  // reference's iteration k + q).
  int lex_hint = 0;  // the previous lexicographic solve's iteration count if it converged, else 0

  // p buffers of every strip := buffer `src_buf`'s contents, or the solve's
  // initial field (src_buf < 0): zero for the cavity (cavity-01.cpp:610-611),
  // the previous pressure for the open cases (channel-01.cpp:636, kept in B_PL)
  void lex_set_both(int src_buf) {
    if (src_buf < 0 && P.case_id != CFD_CAVITY) src_buf = B_PL;
    for (auto& s : S) {
      const size_t bytes = (size_t)s.g.nrows * pitch * sizeof(double);
      for (int b : {0, 1}) {
        if (src_buf < 0) HIPC(hipMemsetAsync(s.b[pbuf(b)], 0, bytes, st));
        else if (pbuf(b) != src_buf) HIPC(hipMemcpyAsync(s.b[pbuf(b)], s.b[src_buf], bytes, hipMemcpyDeviceToDevice, st));
      }
    }
  }
  void lex_reset_tests() {
    HIPC(hipMemsetAsync(lexbits, 0, lexbits_words * sizeof(unsigned long long), st));
    HIPC(hipMemsetAsync(stop, 0, 2 * sizeof(int), st));
    HIPC(hipMemsetAsync(cscr, 0xff, 4 * sizeof(double), st));  // (NaN: no deferred residual pending)
  }
  // the step's corner solid of the final field (lexw.hpp step_corner_kernel)
  void step_corner(int bp) {
    if (P.case_id != CFD_BACKSTEP) return;
    if (multi()) exchange(bp, 1);  // (the corner's south neighbour may sit in a halo row)
    for (auto& s : S) {
      step_corner_kernel<<<1, 64, 0, st>>>(s.g, C, s.b[bp]);
      check_launch("step_corner");
    }
  }
  // replay of k iterations (no tests) from the field in both buffers (base);
  // returns the buffer index (0/1) holding the result
  int lex_replay(int base, int k) {
    if (k <= 0) return base;
    int dc, dk;
    const int n = run_lexw(base, k, false, 1, 0, &dk, &dc, false);
    T.poisson_launches += n;
    T.poisson_sweeps += (long long)n * lexw_ns();
    return (base + n) % 2;
  }

  // On ranks (a strip per process) the same launches run on every rank, the
  // halo rows exchanged before each; the stop rule reads exceedance bits OR-ed
  // over the ranks (lexw_reduce_bits) and every host decision (stop, replay,
  // exact fallback) derives from all-reduced values, so all ranks take the
  // same path and issue the same RCCL sequence.
  void solve_lexw(cfd_step_info* out) {
    const int ns = lexw_ns();
    const int K = P.max_iters;
    const int base = pcur & 1;
    // the initial field in both buffers (cells not yet started are read from
    // either): zero for the cavity (cavity-01.cpp:610-611); the open cases start
    // from the previous pressure (channel-01.cpp:636), saved in B_PL for replays
    if (P.case_id != CFD_CAVITY)
      for (auto& s : S)
        HIPC(hipMemcpyAsync(s.b[B_PL], s.b[pbuf(base)], (size_t)s.g.nrows * pitch * sizeof(double),
                            hipMemcpyDeviceToDevice, st));
    lex_set_both(-1);
    solve_tolerance();
    if (multi()) exchange(B_F, HALO - 1);
    // bit of iteration k: k + offset; waves touch iterations from about
    // -(nx+ny)/2 (cells not yet started) to K + (nx+ny)/2 (cells finished)
    const size_t words = (size_t)LEXW_SHARDS * ((lexw_offset() + K + (P.nx + P.ny) / 2 + 256) / 64 + 2);
    if (lexbits_words < words) {
      if (lexbits) HIPC(hipFree(lexbits));
      lexbits = nullptr;
      HIPC(hipMalloc(&lexbits, words * sizeof(unsigned long long)));
      lexbits_words = words;
    }
    if (ranks() && lexflags_n < (size_t)K + 1) {
      if (lexflags) HIPC(hipFree(lexflags));
      lexflags = nullptr;
      HIPC(hipMalloc(&lexflags, ((size_t)K + 1) * sizeof(double)));
      lexflags_n = (size_t)K + 1;
    }
    lex_reset_tests();
    HIPC(hipEventRecord(ev_a, st));
    const int kexact = (ns < 3) ? 1 : (lex_hint > 0 && lex_hint < K) ? std::max(1, lex_hint - 64) : K;
    int iters = K, kstop = -1, code = 0, fin = base;
    if (K > 0) {
      const int launched = run_lexw(base, K, true, kexact, 0, &kstop, &code, true);
      fin = (base + launched) % 2;
      T.poisson_launches += launched;
      T.poisson_sweeps += (long long)launched * ns;
    } else {
      kstop = 0;
      code = 1;
    }
    double res = -1.0;  // (< 0: recompute from the final field)
    if (code == 1) {  // the reference stops at kstop < K: every cell redoes exactly kstop iterations
      iters = kstop;
      lex_set_both(-1);
      fin = lex_replay(base, kstop);
    } else if (code == 2) {  // kstop left open by the sampled rows: rebuild its field, evaluate it exactly
      ++T.proof_fallbacks;
      lex_set_both(-1);
      const int b1 = lex_replay(base, kstop);
      step_corner(pbuf(b1));  // (also the continuation's initial field: the refresh after iteration kstop)
      const double rk = final_residual(pbuf(b1));
      double t2[2];
      HIPC(hipMemcpy(t2, tolv, sizeof t2, hipMemcpyDeviceToHost));
      if (!(rk > t2[0])) {  // cavity-01.cpp:635: the loop stops at kstop
        iters = kstop;
        fin = b1;
        res = rk;
      } else {  // continuation from iteration kstop's field (kept in B_P2), every cell evaluated
        for (auto& s : S)
          HIPC(hipMemcpyAsync(s.b[B_P2], s.b[pbuf(b1)], (size_t)s.g.nrows * pitch * sizeof(double),
                              hipMemcpyDeviceToDevice, st));
        lex_set_both(pbuf(b1));
        lex_reset_tests();
        int k2 = -1, code2 = 0;
        const int n3 = run_lexw(b1, K - kstop, true, 1, 1, &k2, &code2, false);
        T.poisson_launches += n3;
        T.poisson_sweeps += (long long)n3 * ns;
        if (code2 == 1) {  // stops at kstop + k2 (< K): redo k2 iterations from kstop's field
          iters = kstop + k2;
          lex_set_both(B_P2);
          fin = lex_replay(b1, k2);
        } else {
          iters = K;
          fin = (b1 + n3) % 2;
        }
      }
    }
    HIPC(hipEventRecord(ev_b, st));
    // the reported residual: max-norm of the final field (cavity-01.cpp:659-677)
    if (iters == 0) {
      double t2[2];
      HIPC(hipMemcpyAsync(t2, tolv, sizeof t2, hipMemcpyDeviceToHost, st));
      HIPC(hipStreamSynchronize(st));
      res = t2[1];
    } else if (res < 0.0) {
      step_corner(pbuf(fin));
      res = final_residual(pbuf(fin));
    }
    HIPC(hipEventSynchronize(ev_b));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
    T.poisson_ms += ms;
    long long owned = 0;
    for (auto& s : S) owned += (long long)(s.g.j1 - s.g.j0 + 1) * P.nx;
    T.poisson_cell_updates += owned * iters;
    pcur = fin;
    lex_hint = (iters < K) ? iters : 0;
    if (out) {
      out->sor_iterations = iters;
      out->residual = res;
    }
  }

  // red-black solve of a reference-sized grid in one persistent workgroup
  // (small.hpp): one strip, no ranks, p fits the LDS (small_solve = CFD_OFF: never)
  bool use_small() const {
    return P.small_solve != CFD_OFF && P.ordering == CFD_ORDER_RB && S.size() == 1 && !comm &&
           (long long)(P.nx + 2) * (P.ny + 2) <= SMALL_CELLS;
  }

  void solve_small(cfd_step_info* out) {
    Strip& s = S[0];
    double* X = s.b[pbuf(pcur)];
    if (P.case_id == CFD_CAVITY)  // cavity-01.cpp:610-611: each solve starts from a zero field
      HIPC(hipMemsetAsync(X, 0, (size_t)s.g.nrows * pitch * sizeof(double), st));
    solve_tolerance();
    int* d_it = stop;
    double* d_res = total + 2;
    HIPC(hipEventRecord(ev_a, st));
    const int ce = std::max(1, P.check_every);
    const long long per_colour = ((long long)P.nx * P.ny + 1) / 2;
    const int maxc = per_colour <= 2 * SMALL_THREADS ? 2 : per_colour <= 4 * SMALL_THREADS ? 4
                   : per_colour <= 8 * SMALL_THREADS ? 8 : SMALL_MAXC;
#define CFD_SMALL_LAUNCH(CASE)                                                                                    \
  if (maxc == 2)                                                                                                  \
    poisson_small_kernel<CASE, 2><<<1, SMALL_THREADS, 0, st>>>(s.g, C, X, s.b[B_F], tolv, P.max_iters, ce, d_it, d_res); \
  else if (maxc == 4)                                                                                             \
    poisson_small_kernel<CASE, 4><<<1, SMALL_THREADS, 0, st>>>(s.g, C, X, s.b[B_F], tolv, P.max_iters, ce, d_it, d_res); \
  else if (maxc == 8)                                                                                             \
    poisson_small_kernel<CASE, 8><<<1, SMALL_THREADS, 0, st>>>(s.g, C, X, s.b[B_F], tolv, P.max_iters, ce, d_it, d_res); \
  else                                                                                                            \
    poisson_small_kernel<CASE, SMALL_MAXC><<<1, SMALL_THREADS, 0, st>>>(s.g, C, X, s.b[B_F], tolv, P.max_iters, ce, d_it, d_res)
    if (P.case_id == CFD_CAVITY) { CFD_SMALL_LAUNCH(CAVITY); }
    else if (P.case_id == CFD_CHANNEL) { CFD_SMALL_LAUNCH(CHANNEL); }
    else { CFD_SMALL_LAUNCH(BACKSTEP); }
#undef CFD_SMALL_LAUNCH
    check_launch("poisson_small");
    HIPC(hipEventRecord(ev_b, st));
    int iters = 0;
    double res = 0;
    HIPC(hipMemcpyAsync(&iters, d_it, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(&res, d_res, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
    T.poisson_ms += ms;
    T.poisson_launches += 1;
    T.poisson_sweeps += iters;
    T.poisson_cell_updates += (long long)P.nx * P.ny * iters;
    if (out) {
      out->sor_iterations = iters;
      out->residual = res;
    }
  }

  // max-norm residual of the cavity field in p buffer `bp` (cavity-01.cpp:659-677)
  double final_residual(int bp) {
    if (multi()) exchange(bp, 1);
    HIPC(hipMemsetAsync(resmax, 0, RES_SHARDS * SHARD_STRIDE * sizeof(double), st));
    for (auto& s : S) {
      if (P.case_id == CFD_CAVITY) {
        cavity_resmax_kernel<<<pair_grid(s), 256, 0, st>>>(s.g, C, s.b[bp], s.b[B_F], resmax);
      } else {
        const int rows = std::min(s.g.j1, P.ny) - std::max(s.g.j0, 1) + 1;
        const dim3 grid((P.nx + 63) / 64, std::max(1, (rows + 3) / 4));
        if (P.case_id == CFD_CHANNEL) open_resmax_kernel<CHANNEL><<<grid, 256, 0, st>>>(s.g, C, s.b[bp], s.b[B_F], resmax);
        else open_resmax_kernel<BACKSTEP><<<grid, 256, 0, st>>>(s.g, C, s.b[bp], s.b[B_F], resmax);
      }
      check_launch("resmax");
    }
    if (comm && comm->nranks > 1) comm_allreduce_max(comm, resmax, RES_SHARDS * SHARD_STRIDE, st);
    HIPC(hipMemcpyAsync(h_shard, resmax, RES_SHARDS * SHARD_STRIDE * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    double res = 0.0;
    for (int q = 0; q < RES_SHARDS; ++q) res = std::max(res, h_shard[q * SHARD_STRIDE]);
    return res;
  }

  // the reference order on a reference-sized grid in one workgroup (smlex.hip):
  // one strip, no ranks, p fits the LDS twice (small_solve = CFD_OFF: never)
  double* smlex_ck = nullptr;  // its checkpoints (smlex_ck_doubles)
  bool use_smlex() const {
    return P.ordering == CFD_ORDER_LEX && P.small_solve != CFD_OFF && S.size() == 1 && !comm && smlex_fits(S[0].g, C);
  }

  void solve_smlex(cfd_step_info* out) {
    Strip& s = S[0];
    double* X = s.b[pbuf(pcur)];
    if (P.case_id == CFD_CAVITY)  // cavity-01.cpp:610-611: each solve starts from a zero field
      HIPC(hipMemsetAsync(X, 0, (size_t)s.g.nrows * pitch * sizeof(double), st));
    if (!smlex_ck)
      HIPC(hipMalloc(&smlex_ck, smlex_ck_doubles(P.nx, P.ny) * sizeof(double)));
    solve_tolerance();
    int* d_it = stop;
    double* d_res = total + 2;
    HIPC(hipEventRecord(ev_a, st));
    smlex_launch(P.case_id, s.g, C, X, s.b[B_F], tolv, P.max_iters, smlex_ck, d_it, d_res, st);
    check_launch("poisson_smlex");
    HIPC(hipEventRecord(ev_b, st));
    int iters = 0;
    double res = 0;
    HIPC(hipMemcpyAsync(&iters, d_it, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(&res, d_res, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
    T.poisson_ms += ms;
    T.poisson_launches += 1;
    T.poisson_sweeps += iters;
    T.poisson_cell_updates += (long long)P.nx * P.ny * iters;
    if (out) {
      out->sor_iterations = iters;
      out->residual = res;
    }
  }

  void solve(cfd_step_info* out) {
    if (use_smlex()) {
      T.sor_kernel = CFD_SOR_SMLEX;
      solve_smlex(out);
      return;
    }
    if (res_on && P.ordering == CFD_ORDER_LEX) {
      T.sor_kernel = CFD_SOR_RESIDENT;
      solve_resident_lex_segments(out);  // (an iteration no sample settles: an exact window, then resident again)
      return;
    }
    if (use_lexw()) {
      T.sor_kernel = CFD_SOR_LEXW;
      solve_lexw(out);
      return;
    }
    if (P.ordering == CFD_ORDER_LEX) {
      T.sor_kernel = CFD_SOR_LEX;
      solve_lex(out);
      return;
    }
    if (use_small()) {
      T.sor_kernel = CFD_SOR_SMALL;
      solve_small(out);
      return;
    }
    if (res_on) {
      T.sor_kernel = CFD_SOR_RESIDENT;
      solve_resident_segments(out);  // (an iteration the proof leaves open: an exact window, then resident again)
      return;
    }
    T.sor_kernel = tile_on ? CFD_SOR_TILE : CFD_SOR_MARCH;
    solve_rb(out, 0);
  }

  // A solve on the resident launch, in segments (round 6). A launch that
  // leaves an iteration open hands the next stretch of the solve to the exact
  // launches - a window of RES_WINDOW_LAUNCHES of them from the field reached
  // (red-black: the launch's proven iterations replayed; the reference order:
  // its intact input) - and, unless the reference stops inside the window or
  // at its end, relaunches the resident kernel from the window's field for
  // the rest of the solve. Each segment is a solve from the field it starts
  // with: an SOR sweep depends on nothing but the current field (and the
  // channel's ghosts as stored, which the last sweep's refresh left), and the
  // reference's loop goes on through every iteration before the open one, so
  // the segments' iterations are the reference's, bit for bit. A solve from
  // rest (its first iterations' residuals live at the lid's corners: no proof,
  // no sampled row) thus pays one window, not the whole solve on the exact
  // path (round 5: ~2.3x a later step at 1024^2). After RES_MAX_SEGMENTS
  // windows the exact path finishes the solve.
  static constexpr int RES_WINDOW_LAUNCHES = 32, RES_MAX_SEGMENTS = 8;
  struct CapGuard {  // the segment's iteration cap in P.max_iters (every solve path reads the cap there)
    int& ref;
    int saved;
    CapGuard(int& r, int v) : ref(r), saved(r) { ref = v; }
    ~CapGuard() { ref = saved; }
  };
  double tol_host() {
    double t2[2];
    HIPC(hipMemcpyAsync(t2, tolv, sizeof t2, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    return t2[0];
  }
  int res_segments = 0;  // segments of the last solve (tests: a solve from rest relaunches the resident kernel)
  void solve_resident_segments(cfd_step_info* out) {
    const int K = P.max_iters;
    int kdone = 0;
    cfd_step_info si{0, 0.0};
    res_segments = 0;
    for (int seg = 0;; ++seg) {
      ++res_segments;
      int k0 = 0;
      const long long to0 = T.resident_timeouts;
      bool done;
      {
        CapGuard cg(P.max_iters, K - kdone);
        done = solve_resident(&si, k0, seg == 0);
      }
      if (done) {
        kdone += si.sor_iterations;
        break;
      }
      const bool broken = T.resident_timeouts != to0;  // (not co-resident after all: no relaunch)
      // the field after kdone + k0 iterations: the replay's output (k0 > 0) or the intact input
      if (k0 > 0) pcur = (pcur + 1) % nbufs();
      kdone += k0;
      const bool last = broken || seg + 1 >= RES_MAX_SEGMENTS;
      const int w = last ? K - kdone : std::min(RES_WINDOW_LAUNCHES * sweeps_per_launch(), K - kdone);
      {
        CapGuard cg(P.max_iters, w);
        rb_fresh = false;
        rb_exact = !last;
        solve_rb(&si, 0);
        rb_fresh = true;
        rb_exact = false;
      }
      kdone += si.sor_iterations;
      // the reference stopped inside the window, the cap, or iteration kdone's
      // exact residual (the window's last, which its launches do not test) meets
      // the tolerance: the solve ends here
      if (last || si.sor_iterations < w || kdone >= K || !(si.residual > tol_host())) break;
    }
    if (out) {
      out->sor_iterations = kdone;
      out->residual = si.residual;
    }
  }
  // the reference order: the resident launch's open iteration leaves its
  // input intact; the exact window is the multi-block march from that field
  // (lexw.hpp, every cell's residual evaluated: kexact 1), its stop replayed
  // from the window's initial field (kept in B_P2)
  void solve_resident_lex_segments(cfd_step_info* out) {
    const int K = P.max_iters;
    int kdone = 0;
    cfd_step_info si{0, 0.0};
    double res = 0.0;
    res_segments = 0;
    for (int seg = 0;; ++seg) {
      ++res_segments;
      const long long to0 = T.resident_timeouts;
      bool done;
      {
        CapGuard cg(P.max_iters, K - kdone);
        done = solve_resident_lex(&si, seg == 0);
      }
      if (done) {
        kdone += si.sor_iterations;
        res = si.residual;
        break;
      }
      if (seg == 0 && T.resident_timeouts != to0) {  // (not co-resident: the exact path takes the whole solve)
        solve_lexw(out);
        return;
      }
      const bool last = T.resident_timeouts != to0 || seg + 1 >= RES_MAX_SEGMENTS;
      // (the window reaches past the open iteration: its launches cost the
      // skew's ramps, ~(nx + ny) / 2NS of them, whatever its length)
      const int ko = std::max(1, si.sor_iterations);
      const int w = last ? K - kdone : std::min(std::max(RES_WINDOW_LAUNCHES * 2 * lexw_ns(), ko + 64), K - kdone);
      int k2 = 0;
      const bool stopped = lexw_window(w, &k2, &res);
      kdone += k2;
      if (stopped || last || kdone >= K) break;
    }
    lex_hint = 0;  // (the segments keep no sampled-row hint)
    if (out) {
      out->sor_iterations = kdone;
      out->residual = res;
    }
  }
  // w reference-order iterations from the field in pbuf(pcur & 1) with every
  // cell's residual evaluated; returns true when the reference stops inside
  // the window or at its end (the exact residual of its last iteration), with
  // *k = the iterations run (the field in pbuf(pcur)) and *res that residual
  bool lexw_window(int w, int* k, double* res) {
    const int ns = lexw_ns();
    const int b0 = pcur & 1;
    for (auto& s : S)
      HIPC(hipMemcpyAsync(s.b[B_P2], s.b[pbuf(b0)], (size_t)s.g.nrows * pitch * sizeof(double),
                          hipMemcpyDeviceToDevice, st));
    lex_set_both(B_P2);
    const size_t words = (size_t)LEXW_SHARDS * ((lexw_offset() + w + (P.nx + P.ny) / 2 + 256) / 64 + 2);
    if (lexbits_words < words) {
      if (lexbits) HIPC(hipFree(lexbits));
      lexbits = nullptr;
      HIPC(hipMalloc(&lexbits, words * sizeof(unsigned long long)));
      lexbits_words = words;
    }
    lex_reset_tests();
    HIPC(hipEventRecord(ev_a, st));
    int k2 = -1, code = 0;
    const int n = run_lexw(b0, w, true, 1, 1, &k2, &code, false);
    T.poisson_launches += n;
    T.poisson_sweeps += (long long)n * ns;
    int fin = (b0 + n) % 2, iters = w;
    if (code == 1) {  // the reference stops at k2 < w: redo k2 iterations from the window's field
      iters = k2;
      lex_set_both(B_P2);
      fin = lex_replay(b0, k2);
    }
    HIPC(hipEventRecord(ev_b, st));
    *res = final_residual(pbuf(fin));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
    T.poisson_ms += ms;
    long long owned = 0;
    for (auto& s : S) owned += (long long)(s.g.j1 - s.g.j0 + 1) * P.nx;
    T.poisson_cell_updates += owned * iters;
    pcur = fin;
    *k = iters;
    return code == 1 || !(*res > tol_host());
  }

  // The register-resident solve (resident.hpp): one persistent launch runs the
  // whole capped solve. Returns true when the solve is done; false with k0:
  // iteration k0 + 1's group was left open by the proof, the field after k0
  // iterations is in the output buffer of "launch 0" (pbuf(base + 1)), and
  // solve_rb goes on from there with exact residuals (k0 = 0: from scratch).
  bool solve_resident(cfd_step_info* out, int& k0, bool fresh = true) {
    Strip& s = S[0];
    const int base = pcur;
    const size_t fbytes = (size_t)s.g.nrows * pitch * sizeof(double);
    double* pin = s.b[pbuf(base)];
    double* pout = s.b[pbuf((base + 1) % nbufs())];
    // the cavity starts each solve from a zero field (cavity-01.cpp:610-611),
    // the channel from the previous pressure (channel-01.cpp:636); a later
    // segment of the solve (solve_resident_segments) from the field reached
    if (P.case_id == CFD_CAVITY && fresh) HIPC(hipMemsetAsync(pin, 0, fbytes, st));
    const bool open = P.case_id == CFD_CHANNEL;
    const int cid = open ? CHANNEL : CAVITY;
    solve_tolerance();
    if (!res_x[0])
      for (auto*& x : res_x) {
        HIPC(hipMalloc(&x, fbytes));
        HIPC(hipMemsetAsync(x, 0, fbytes, st));  // (cells outside the grid stay finite)
      }
    const int ntiles = rplan.ctiles * rplan.rtiles, K = P.max_iters;
    const size_t words = res_state_words(ntiles, K);
    if (words > res_state_n) {
      if (res_state) HIPC(hipFree(res_state));
      res_state = nullptr;
      HIPC(hipMalloc(&res_state, words * sizeof(unsigned)));
      res_state_n = words;
    }
    ResCtl R{};
    R.xa = res_x[0];
    R.xb = res_x[1];
    R.flags = res_state;
    R.proven = R.flags + ntiles;
    R.status = reinterpret_cast<int*>(R.proven + K + 1);
    R.tol = tolv;
    R.K = K;
    R.check_every = std::max(1, P.check_every);
    HIPC(hipMemsetAsync(res_state, 0, words * sizeof(unsigned), st));
    HIPC(hipMemsetAsync(R.status, 0xff, sizeof(int), st));  // (-1 until the launch sets its status)
    HIPC(hipEventRecord(ev_a, st));
    res_launch(cid, false, s.g, C, pin, pout, s.b[B_F], R, rplan, 0, st);
    check_launch("poisson (resident)");
    if (open) res_refresh(s.g, pout, st);  // the refresh after the last sweep (its red ghosts)
    HIPC(hipEventRecord(ev_b, st));
    HIPC(hipMemcpyAsync(h_stat, R.status, 3 * sizeof(int), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const int code = h_stat[0], kst = h_stat[1], timeout = h_stat[2];
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
    T.poisson_ms += ms;
    T.poisson_launches += 1;
    // a wait that timed out (tiles not co-resident after all): nothing but the
    // exchange fields and p_out was written, p_in is intact - the exact
    // launches take the whole solve
    if (timeout) {
      ++T.resident_timeouts;
      k0 = 0;
      return false;
    }
    if (code == -1) throw Error(CFD_E_STATE, "resident SOR solve: the launch set no status");
    if (code == 0 || code == 1) {
      const int iters = code == 0 ? K : 0;
      double res;
      if (iters == 0) {
        double t2[2];
        HIPC(hipMemcpy(t2, tolv, sizeof t2, hipMemcpyDeviceToHost));
        res = t2[1];
      } else {
        pcur = (base + 1) % nbufs();
        res = final_residual(pbuf(pcur));  // the final field's (cavity-01.cpp:659-677)
      }
      T.poisson_sweeps += iters;
      T.poisson_cell_updates += (long long)P.nx * P.ny * iters;
      if (out) {
        out->sor_iterations = iters;
        out->residual = res;
      }
      return true;
    }
    if (code != 2 || kst < 0 || kst >= K) throw Error(CFD_E_STATE, "resident SOR solve: bad status");
    ++T.proof_fallbacks;
    k0 = kst;
    if (k0 > 0) {  // the field after k0 iterations, from the solve's intact input
      HIPC(hipMemsetAsync(res_state, 0, words * sizeof(unsigned), st));
      R.K = k0;
      HIPC(hipEventRecord(ev_a, st));
      res_launch(cid, false, s.g, C, pin, pout, s.b[B_F], R, rplan, RES_REPLAY, st);
      check_launch("poisson (resident replay)");
      if (open) res_refresh(s.g, pout, st);
      HIPC(hipEventRecord(ev_b, st));
      HIPC(hipMemcpyAsync(h_stat, R.status, 3 * sizeof(int), hipMemcpyDeviceToHost, st));
      HIPC(hipStreamSynchronize(st));
      HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
      T.poisson_ms += ms;
      T.poisson_launches += 1;
      if (h_stat[2]) {  // (as above: the exact launches from scratch)
        ++T.resident_timeouts;
        k0 = 0;
      }
    }
    return false;
  }

  // The reference's order as one resident launch (resident.hip, LEX): every
  // cell's iterations in the skewed half-sweep order, the stop rule from
  // sampled residuals. Returns false (nothing changed but the tolerance) when
  // an iteration before the cap has no sampled exceedance: it may be the
  // reference's stop, which only the exact evaluation settles (solve_lexw).
  bool solve_resident_lex(cfd_step_info* out, bool fresh = true) {
    Strip& s = S[0];
    const int base = pcur & 1;
    const size_t fbytes = (size_t)s.g.nrows * pitch * sizeof(double);
    double* pin = s.b[pbuf(base)];
    double* pout = s.b[pbuf(base ^ 1)];
    // the cavity starts each solve from a zero field (cavity-01.cpp:610-611);
    // the channel from the previous pressure (channel-01.cpp:636), left intact in
    // p_in for the exact path; a later segment from the field reached
    if (P.case_id == CFD_CAVITY && fresh) HIPC(hipMemsetAsync(pin, 0, fbytes, st));
    solve_tolerance();
    if (!res_x[0])
      for (auto*& x : res_x) {
        HIPC(hipMalloc(&x, fbytes));
        HIPC(hipMemsetAsync(x, 0, fbytes, st));
      }
    const int ntiles = rplan.ctiles * rplan.rtiles, K = P.max_iters;
    const size_t words = res_state_words(ntiles, K);
    if (words > res_state_n) {
      if (res_state) HIPC(hipFree(res_state));
      res_state = nullptr;
      HIPC(hipMalloc(&res_state, words * sizeof(unsigned)));
      res_state_n = words;
    }
    const int bwords = res_lex_words(P.nx, P.ny, K);
    const size_t bn = (size_t)8 * bwords;
    if (bn > res_bits_n) {
      if (res_bits) HIPC(hipFree(res_bits));
      res_bits = nullptr;
      HIPC(hipMalloc(&res_bits, bn * sizeof(unsigned long long)));
      res_bits_n = bn;
    }
    ResCtl R{};
    R.xa = res_x[0];
    R.xb = res_x[1];
    R.flags = res_state;
    R.proven = R.flags + ntiles;
    R.status = reinterpret_cast<int*>(R.proven + K + 1);
    R.tol = tolv;
    R.K = K;
    R.check_every = std::max(1, P.check_every);
    R.bits = res_bits;
    R.bwords = bwords;
    R.koff = res_lex_koff(P.nx, P.ny);
    HIPC(hipMemsetAsync(res_state, 0, words * sizeof(unsigned), st));
    HIPC(hipMemsetAsync(res_bits, 0, bn * sizeof(unsigned long long), st));
    HIPC(hipMemsetAsync(R.status, 0xff, sizeof(int), st));  // (-1 until the launch sets its status)
    HIPC(hipEventRecord(ev_a, st));
    res_launch(P.case_id == CFD_CHANNEL ? CHANNEL : CAVITY, true, s.g, C, pin, pout, s.b[B_F], R, rplan, 0, st);
    check_launch("poisson (resident, reference order)");
    HIPC(hipEventRecord(ev_b, st));
    HIPC(hipMemcpyAsync(h_stat, R.status, 3 * sizeof(int), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    const int code = h_stat[0], timeout = h_stat[2];
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
    T.poisson_ms += ms;
    T.poisson_launches += 1;
    if (timeout) {  // (tiles not co-resident after all: p_in is intact, the exact path takes the solve)
      ++T.resident_timeouts;
      return false;
    }
    if (code == 2) {
      ++T.proof_fallbacks;
      if (out) out->sor_iterations = h_stat[1];  // (the open iteration)
      return false;
    }
    if (code != 0 && code != 1) throw Error(CFD_E_STATE, "resident SOR solve: bad status");
    const int iters = code == 0 ? K : 0;
    double res;
    if (iters == 0) {
      double t2[2];
      HIPC(hipMemcpy(t2, tolv, sizeof t2, hipMemcpyDeviceToHost));
      res = t2[1];
      pcur = base;
    } else {
      pcur = base ^ 1;
      res = final_residual(pbuf(pcur));  // the final field's (cavity-01.cpp:659-677)
    }
    T.poisson_sweeps += iters;
    T.poisson_cell_updates += (long long)P.nx * P.ny * iters;
    if (out) {
      out->sor_iterations = iters;
      out->residual = res;
    }
    return true;
  }

  // The red-black solve as a sequence of launches (march or LDS tiles). k0 > 0:
  // iterations 1 .. k0 are done (solve_resident) and every one of them was
  // proven to go on; their field is launch 0's output, and the solve goes on
  // from there with one chunk of exact launches first.
  bool rb_fresh = true;     // solve_rb starts a solve (the cavity's zero field); false: a segment from the field in pcur
  bool rb_exact = false;    // solve_rb: exact residuals in every launch (the window after a resident launch's open iteration)
  void solve_rb(cfd_step_info* out, int k0) {
    const int base = pcur;
    HIPC(hipMemsetAsync(ring, 0, (size_t)RING * RES_SHARDS * SHARD_STRIDE * sizeof(double), st));
    HIPC(hipMemsetAsync(stop, 0, 2 * sizeof(int), st));
    if (P.case_id == CFD_CAVITY && k0 == 0 && rb_fresh) {
      // cavity-01.cpp:610-611: each solve starts from a zero field
      for (auto& s : S)
        HIPC(hipMemsetAsync(s.b[pbuf(base)], 0, (size_t)s.g.nrows * pitch * sizeof(double), st));
    }
    solve_tolerance();
    if (multi()) exchange(B_F, HALO - 1);
    // Launch plan: spl iterations per launch (3 for the cavity, 2 otherwise,
    // 1 with sweeps_per_launch = 1 or a legacy kernel), a shorter last launch
    // for the remainder. Launch m reads buffer (base+m) mod nbufs and tests the
    // iterations of launch m-1 (lagged: m-2); iteration 0 = initial residual.
    const int spl = sweeps_per_launch();
    const int chunk = P.chunk > 0 ? P.chunk : 32;  // launches between host polls
    const int lag = lagged() ? 1 : 0;
    launches.clear();
    ar_pending = {0, 0};
    HIPC(hipEventRecord(ev_a, st));
    int k = 0, c = 0, m = 0;
    int last_tested = -1;  // highest iteration some launch tests
    // Proof mode (cavity 3/4-sweep launches): windows test proof ratios. An
    // iteration the proof leaves open restarts the solve at the launch that
    // computed it (its input is intact: later launches exited at entry), with
    // exact launches for one chunk, then proof mode again; windows over the
    // launches before it are empty (every one of their iterations was proven
    // to go on). Each launch record says which kind of value its slots hold.
    int proof_from = (proof_ok() && !rb_exact) ? 0 : INT32_MAX;  // first launch (index) in proof mode
    int exact_from = 0;  // first launch whose iterations later launches test
    int iters = 0;
    if (k0 > 0) {  // "launch 0" = the resident solve's iterations 1 .. k0 (all proven to go on)
      launches.push_back({1, k0, true});
      k = k0;
      m = 1;
      exact_from = 1;
      last_tested = k0;
      if (proof_from == 0) proof_from = 1 + chunk;
    }
    auto launch_of = [&](int kk) {
      for (size_t q = 0; q < launches.size(); ++q)
        if (kk >= launches[q].first && kk <= launches[q].first + launches[q].n - 1) return (int)q;
      throw Error(CFD_E_STATE, "iteration outside the launches of this solve");
    };
    for (;;) {
      bool stopped = false;
      while (k < P.max_iters && !stopped) {
        for (int j = 0; j < chunk && k < P.max_iters; ++j, ++m) {
          const bool proof = m >= proof_from;
          const int n = std::min((proof && !tile_on) ? proof_ns : spl, P.max_iters - k);  // (tiles: spl either way)
          const int src = m - 1 - lag;
          int ka = 1, kb = 0;  // empty window
          window_proof = false;
          if (src >= exact_from) {
            ka = launches[src].first;
            kb = ka + launches[src].n - 1;
            window_proof = launches[src].proof;
          } else if (src == -1) {
            ka = kb = 0;
          }
          proof_launch = proof && (n >= 3 || tile_on);
          poisson_launch(m, k + 1, n, base, ka, kb, false);
          if (ka <= kb) last_tested = std::max(last_tested, kb);
          launches.push_back({k + 1, n, proof_launch});
          k += n;
        }
        join_b();
        HIPC(hipMemcpyAsync(h_stat + 2 * (c & 1), stop, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
        HIPC(hipEventRecord(ev_poll[c & 1], st));
        if (c > 0) {
          HIPC(hipEventSynchronize(ev_poll[(c - 1) & 1]));
          if (h_stat[2 * ((c - 1) & 1)] != 0) stopped = true;
        }
        ++c;
      }
      flush_allreduce(st);  // overlapped launches all-reduce one launch late: the last one
      int code = 0, kstop = 0;
      if (c > 0) {
        HIPC(hipEventSynchronize(ev_poll[(c - 1) & 1]));
        const int* hs = h_stat + 2 * ((c - 1) & 1);
        code = hs[0];
        kstop = hs[1];
      }
      iters = (code == 1) ? kstop : P.max_iters;
      int open_k = (code == 2) ? kstop : -1;  // an iteration the proof left open
      // iterations after the last one a launch tested (the last launch(es), and
      // the initial residual if no launch tested it): tested here, in order (the
      // reference's while condition, cavity-01.cpp:633)
      if (code == 0 && last_tested < P.max_iters - 1) {
        HIPC(hipStreamSynchronize(st));
        double t2[2];
        HIPC(hipMemcpy(t2, tolv, sizeof t2, hipMemcpyDeviceToHost));
        for (int kk = last_tested + 1; kk <= P.max_iters - 1; ++kk) {
          double r;
          bool pr = false;
          if (kk == 0) {
            r = t2[1];
          } else if (kk % P.check_every == 0) {
            const double* slot = ring + (size_t)(kk & (RING - 1)) * RES_SHARDS * SHARD_STRIDE;
            HIPC(hipMemcpy(h_shard, slot, RES_SHARDS * SHARD_STRIDE * sizeof(double), hipMemcpyDeviceToHost));
            r = 0.0;
            for (int q = 0; q < RES_SHARDS; ++q) r = std::max(r, h_shard[q * SHARD_STRIDE]);
            pr = launches[launch_of(kk)].proof;
          } else {
            continue;
          }
          if (pr) {
            if (!(r > 1.0)) {
              open_k = kk;
              break;
            }
          } else if (!(r > t2[0])) {
            iters = kk;
            break;
          }
        }
      }
      if (open_k < 0) break;
      // exact evaluation from the launch that computed open_k
      join_b();
      HIPC(hipStreamSynchronize(st));
      if (st_b) HIPC(hipStreamSynchronize(st_b));
      const int L = launch_of(open_k);
      k = launches[L].first - 1;
      m = L;
      launches.resize(L);
      last_tested = k;
      exact_from = L;
      proof_from = L + chunk;
      c = 0;  // the polls so far are stale (stop code 2): the next chunk starts a fresh sequence
      ++T.proof_fallbacks;
      HIPC(hipMemsetAsync(ring, 0, (size_t)RING * RES_SHARDS * SHARD_STRIDE * sizeof(double), st));
      HIPC(hipMemsetAsync(stop, 0, 2 * sizeof(int), st));
    }
    proof_launch = window_proof = false;
    HIPC(hipEventRecord(ev_b, st));
    HIPC(hipEventSynchronize(ev_b));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_a, ev_b));
    // the launch that computed iteration `iters`; if it ran further, redo the
    // first r of its iterations from its (intact) input into its output buffer
    int last = -1, replayed = 0;
    long long work_sweeps = 0;
    if (iters > 0) {
      for (size_t q = 0; q < launches.size(); ++q) {
        work_sweeps += launches[q].n;
        if (iters <= launches[q].first + launches[q].n - 1) {
          last = (int)q;
          break;
        }
      }
      const int r = iters - launches[last].first + 1;
      if (r < launches[last].n) {
        HIPC(hipEventRecord(ev_a, st));
        poisson_launch(last, launches[last].first, r, base, 1, 0, true);
        HIPC(hipEventRecord(ev_b, st));
        HIPC(hipEventSynchronize(ev_b));
        float ms2 = 0.f;
        HIPC(hipEventElapsedTime(&ms2, ev_a, ev_b));
        ms += ms2;
        replayed = r;
      }
    }
    // launches that did work (later ones in the enqueued chunks exit at entry)
    T.poisson_ms += ms;
    T.poisson_launches += (last + 1) + (replayed ? 1 : 0);
    T.poisson_sweeps += work_sweeps + replayed;
    T.poisson_overlapped += n_overlapped;
    n_overlapped = 0;
    long long owned = 0;
    for (auto& s : S) owned += (long long)(s.g.j1 - s.g.j0 + 1) * P.nx;
    T.poisson_cell_updates += owned * iters;
    double res;
    if (iters == 0) {
      double t2[2];
      HIPC(hipMemcpy(t2, tolv, sizeof t2, hipMemcpyDeviceToHost));
      res = t2[1];
    } else if (launches[last].proof) {
      // a proof-mode launch computed the last iteration (the cap): the
      // reported residual is the final field's (cavity-01.cpp:659-677)
      res = final_residual(pbuf((base + last + 1) % nbufs()));
    } else {
      const double* slot = ring + (size_t)(iters & (RING - 1)) * RES_SHARDS * SHARD_STRIDE;
      HIPC(hipMemcpy(h_shard, slot, RES_SHARDS * SHARD_STRIDE * sizeof(double), hipMemcpyDeviceToHost));
      res = 0.0;
      for (int q = 0; q < RES_SHARDS; ++q) res = std::max(res, h_shard[q * SHARD_STRIDE]);
    }
    // launch m's output is buffer (base+m+1) mod nbufs (the replay writes there too)
    pcur = (base + last + 1) % nbufs();
    if (out) {
      out->sor_iterations = iters;
      out->residual = res;
    }
  }

  void correct() {
    const int bp = pbuf(pcur);
    if (multi()) exchange(bp, 1);
    for (auto& s : S) {
      correct_kernel<<<s.grid2d, 256, 0, st>>>(s.g, C, s.b[bp], s.b[B_US], s.b[B_VS], s.b[B_U], s.b[B_V]);
      check_launch("correct");
    }
  }

  // run() loop body: cavity-01.cpp:387-390; channel-01.cpp:368-375.
  // adds the last timed step's device time to T.step_ms (waits for it)
  void flush_step_time() {
    if (!step_timed) return;
    HIPC(hipEventSynchronize(ev_s1));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ev_s0, ev_s1));
    T.step_ms += ms;
    step_timed = false;
  }

  void step(cfd_step_info* out) {
    flush_step_time();
    HIPC(hipEventRecord(ev_s0, st));
    if (P.case_id == CFD_CAVITY) {
      apply_bc(false);
      compute_tentative();
      if (thermal) advance_temperature();
      build_source();
      solve(out);
      correct();
    } else {
      compute_tentative();
      apply_bc(true);
      build_source();
      solve(out);
      correct();
      apply_bc(false);
    }
    HIPC(hipEventRecord(ev_s1, st));
    step_timed = true;
    T.steps += 1;
  }

  void stats(cfd_stats* out) {
    if (multi()) exchange(B_V, 1);
    HIPC(hipMemsetAsync(divmax, 0, RES_SHARDS * SHARD_STRIDE * sizeof(double), st));
    for (auto& s : S) {
      centers_stats_kernel<<<s.grid2d, 256, 0, st>>>(s.g, C, s.b[B_U], s.b[B_V], s.b[B_UC], s.b[B_VC],
                                                       partials + s.part_off, divmax);
      check_launch("centers_stats");
    }
    if (P.ordering == CFD_ORDER_LEX && ranks())
      seq_sum_ranks(B_UC, B_VC, 1, total + 1);
    else if (P.ordering == CFD_ORDER_LEX)
      for (size_t q = 0; q < S.size(); ++q)
        seq_sum(S[q], S[q].b[B_UC], S[q].b[B_VC], 1, total + 1, q > 0);
    else
      sum_partials_kernel<<<1, 256, 0, st>>>(partials, (int)npart, total + 1);
    check_launch("sum_partials");
    if (ranks()) {
      if (P.ordering != CFD_ORDER_LEX) comm_allreduce_sum(comm, total + 1, 1, st);
      comm_allreduce_max(comm, divmax, RES_SHARDS * SHARD_STRIDE, st);
    }
    double ke = 0;
    HIPC(hipMemcpyAsync(h_shard, divmax, RES_SHARDS * SHARD_STRIDE * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(&ke, total + 1, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    double md = 0;
    for (int q = 0; q < RES_SHARDS; ++q) md = std::max(md, h_shard[q * SHARD_STRIDE]);
    if (out) {
      out->max_divergence = md;
      out->avg_kinetic_energy = ke / fluid_count;
    }
  }

  // ------------------------------------------------------ field access --
  int field_buf(int field) const {
    switch (field) {
      case CFD_FIELD_P: return pbuf(pcur);
      case CFD_FIELD_SRC: return B_F;
      case CFD_FIELD_US: return B_US;
      case CFD_FIELD_VS: return B_VS;
      case CFD_FIELD_U: return B_U;
      case CFD_FIELD_V: return B_V;
      case CFD_FIELD_UC: return B_UC;
      case CFD_FIELD_VC: return B_VC;
      case CFD_FIELD_T:
        if (thermal) return tcur;
        break;
    }
    throw Error(CFD_E_ARG, "unknown field");
  }
  void field_dims(int field, int& rows, int& cols) const {
    rows = P.ny + 2;
    cols = P.nx + 2;
    if (field == CFD_FIELD_U || field == CFD_FIELD_US) cols = P.nx + 1;
    if (field == CFD_FIELD_V || field == CFD_FIELD_VS) rows = P.ny + 1;
  }
  // rows of `field` stored by this solver: [first, last] (global)
  void owned_field_rows(int field, int& first, int& last) const {
    int rows, cols;
    field_dims(field, rows, cols);
    first = S.front().g.wj0;
    last = std::min(S.back().g.wj1, rows - 1);
  }

  void transfer(int field, double* host, const double* chost, size_t count) {
    int rows, cols, first, last;
    field_dims(field, rows, cols);
    owned_field_rows(field, first, last);
    if (count != (size_t)(last - first + 1) * cols) throw Error(CFD_E_ARG, "host buffer size does not match field shape");
    const int b = field_buf(field);
    if (chost && b == B_F) srcmax_ready = false;  // a new source from the host
    // a pressure from the host goes to every p buffer: cells no launch ever
    // writes (the step block's interior, skipped by the marches) must hold the
    // same value in each, as the reference's single array holds it
    const int nb = (chost && field == CFD_FIELD_P) ? nbufs() : 1;
    for (auto& s : S) {
      const int r0 = s.g.wj0, r1 = std::min(s.g.wj1, rows - 1);
      if (r1 < r0) continue;
      const size_t hoff = (size_t)(r0 - first) * cols;
      for (int q = 0; q < nb; ++q) {
        double* dev = s.b[nb > 1 ? pbuf(q) : b] + (size_t)(r0 - s.g.row_lo) * pitch;
        if (host)
          HIPC(hipMemcpy2DAsync(host + hoff, cols * sizeof(double), dev, pitch * sizeof(double), cols * sizeof(double),
                                r1 - r0 + 1, hipMemcpyDeviceToHost, st));
        else
          HIPC(hipMemcpy2DAsync(dev, pitch * sizeof(double), chost + hoff, cols * sizeof(double), cols * sizeof(double),
                                r1 - r0 + 1, hipMemcpyHostToDevice, st));
      }
    }
    HIPC(hipStreamSynchronize(st));
  }

  void write_vtk(const std::string& fn, double t) {
    if (comm && comm->nranks > 1) throw Error(CFD_E_STATE, "cfd_write_vtk needs the whole grid (single-rank solver)");
    cfd_stats tmp;
    stats(&tmp);  // refreshes the cell-centre fields
    const size_t n = (size_t)(P.ny + 2) * (P.nx + 2);
    std::vector<double> uc(n), vc(n), pr(n);
    transfer(CFD_FIELD_UC, uc.data(), nullptr, n);
    transfer(CFD_FIELD_VC, vc.data(), nullptr, n);
    transfer(CFD_FIELD_P, pr.data(), nullptr, n);
    if (thermal) {
      std::vector<double> tf(n);
      transfer(CFD_FIELD_T, tf.data(), nullptr, n);
      cfd_params q = P;
      q.case_id = CFD_RAYLEIGH_BENARD;
      write_vtk_arrays(q, fn, t, uc.data(), vc.data(), pr.data(), tf.data());
      return;
    }
    write_vtk_arrays(P, fn, t, uc.data(), vc.data(), pr.data());
  }
};

}  // namespace cfd

// =================================================================== C-ABI ==

using cfd::Error;
using cfd::Solver;

struct cfd_solver {
  Solver* impl;
};

template <class F>
static int guard(F&& f) {
  try {
    f();
    return CFD_OK;
  } catch (const Error& e) {
    cfd::set_last_error(e.what());
    return e.code;
  } catch (const std::exception& e) {
    cfd::set_last_error(e.what());
    return CFD_E_DEVICE;
  } catch (...) {
    cfd::set_last_error("unknown error");
    return CFD_E_DEVICE;
  }
}

static Solver* S_(cfd_solver* s) {
  if (!s || !s->impl) throw Error(CFD_E_ARG, "null solver");
  HIPC(hipSetDevice(s->impl->dev));
  return s->impl;
}

extern "C" {

int cfd_abi_version(void) { return CFD_AMD_ABI_VERSION; }
const char* cfd_last_error(void) { return cfd::g_last_error.c_str(); }

cfd_solver* cfd_create(const cfd_params* p, int device, int n_strips) {
  cfd_solver* out = nullptr;
  guard([&] {
    if (!p) throw Error(CFD_E_ARG, "null params");
    if (n_strips < 1) throw Error(CFD_E_ARG, "n_strips must be >= 1");
    if (p->ny < n_strips * cfd::HALO) throw Error(CFD_E_ARG, "each strip needs at least 8 rows (the SOR halo depth)");
    std::vector<std::pair<int, int>> rows;
    for (int k = 0; k < n_strips; ++k) {
      const int a = 1 + (int)((long long)p->ny * k / n_strips);
      const int b = (int)((long long)p->ny * (k + 1) / n_strips);
      rows.emplace_back(a, b);
    }
    out = new cfd_solver{new Solver(*p, device, rows, nullptr)};
  });
  return out;
}

cfd_solver* cfd_create_rank(const cfd_params* p, int device, int row_begin, int row_end, void* comm) {
  cfd_solver* out = nullptr;
  guard([&] {
    if (!p) throw Error(CFD_E_ARG, "null params");
    // (Solver::validate: the one-workgroup reference-order kernel of a thin step block needs one strip)
    if (p->ordering == CFD_ORDER_LEX && p->case_id == CFD_BACKSTEP &&
        !(p->step_i >= 2 && p->inlet_jmax >= 1 && p->inlet_jmax <= p->ny - 2))
      throw Error(CFD_E_ARG, "lexicographic ordering of a backwards step with a block under 2 cells wide or high "
                             "runs on one strip (n_strips = 1, no ranks)");
    if (row_begin < 1 || row_end > p->ny || row_end - row_begin + 1 < cfd::HALO)
      throw Error(CFD_E_ARG, "rank rows must lie in [1, ny] and span at least 8 rows (the SOR halo depth)");
    // the halo exchange talks to ranks rank-1 (rows below) and rank+1 (rows
    // above): ranks must own consecutive row blocks in rank order
    if (auto* cm = static_cast<cfd::Comm*>(comm)) {
      if ((cm->rank == 0) != (row_begin == 1) || (cm->rank == cm->nranks - 1) != (row_end == p->ny))
        throw Error(CFD_E_ARG, "rank rows do not match the communicator rank (rank 0 must own row 1, the last "
                               "rank row ny, ranks in row order)");
    }
    out = new cfd_solver{new Solver(*p, device, {{row_begin, row_end}}, static_cast<cfd::Comm*>(comm))};
  });
  return out;
}

int cfd_destroy(cfd_solver* s) {
  return guard([&] {
    if (!s) return;
    delete s->impl;
    delete s;
  });
}

int cfd_apply_bc(cfd_solver* s) { return guard([&] { S_(s)->apply_bc(false); }); }
int cfd_apply_tentative_bc(cfd_solver* s) { return guard([&] { S_(s)->apply_bc(true); }); }
int cfd_compute_tentative(cfd_solver* s) { return guard([&] { S_(s)->compute_tentative(); }); }
int cfd_advance_temperature(cfd_solver* s) { return guard([&] { S_(s)->advance_temperature(); }); }
int cfd_build_source(cfd_solver* s) { return guard([&] { S_(s)->build_source(); }); }
int cfd_solve_pressure(cfd_solver* s, cfd_step_info* out) { return guard([&] { S_(s)->solve(out); }); }
int cfd_apply_correction(cfd_solver* s) { return guard([&] { S_(s)->correct(); }); }
int cfd_step(cfd_solver* s, cfd_step_info* out) { return guard([&] { S_(s)->step(out); }); }
int cfd_run_steps(cfd_solver* s, int n, cfd_step_info* last) {
  return guard([&] {
    Solver* v = S_(s);
    cfd_step_info info{0, 0.0};
    for (int k = 0; k < n; ++k) v->step(&info);
    if (last) *last = info;
  });
}
int cfd_compute_stats(cfd_solver* s, cfd_stats* out) { return guard([&] { S_(s)->stats(out); }); }

int cfd_field_shape(const cfd_solver* s, int field, int* rows, int* cols) {
  return guard([&] {
    if (!s || !s->impl || !rows || !cols) throw Error(CFD_E_ARG, "null argument");
    int r, c, first, last;
    s->impl->field_dims(field, r, c);
    s->impl->owned_field_rows(field, first, last);
    *rows = last - first + 1;
    *cols = c;
  });
}

int cfd_get_field(cfd_solver* s, int field, double* host, size_t count) {
  return guard([&] {
    if (!host) throw Error(CFD_E_ARG, "null host buffer");
    S_(s)->transfer(field, host, nullptr, count);
  });
}

#if CFD_LEXW_STAMPS
// diagnostic build only: per reference-order launch (H0 / 2NS) and march path,
// {max, sum of wave cycles, waves} (lexw.hpp lexw_stamp_buf), accumulated since
// the library loaded
extern "C" int cfd_lexw_stamps(unsigned long long* out, int n) {
  if (n > cfd::LEXW_STAMP_LAUNCHES * 8 * 3) n = cfd::LEXW_STAMP_LAUNCHES * 8 * 3;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(cfd::lexw_stamp_buf), (size_t)n * 8) == hipSuccess ? n : -1;
}
// per-wave records of a window of launches (lexw.hpp lexw_wstamp_buf)
extern "C" int cfd_lexw_wstamps(unsigned long long* out, int n) {
  if (n > cfd::LEXW_WSTAMP_N * cfd::LEXW_WSTAMP_T * 4) n = cfd::LEXW_WSTAMP_N * cfd::LEXW_WSTAMP_T * 4;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(cfd::lexw_wstamp_buf), (size_t)n * 8) == hipSuccess ? n : -1;
}
#endif

#ifdef CFD_SEQ_STAMPS
// diagnostic build only: seq_walk_kernel's phase ticks (100 MHz) since the last
// call {batch loads, run records, single records, staging, plain chains}
extern "C" int cfd_seq_stamps(cfd_solver* s, int* out) {
  Solver* v = s->impl;
  if (hipStreamSynchronize(v->st) != hipSuccess) return -1;
  if (hipMemcpy(out, v->seqcnt + 1, 5 * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return hipMemset(v->seqcnt + 1, 0, 5 * sizeof(int)) == hipSuccess ? 5 : -1;
}
#endif

#if CFD_MARCH_STAMPS
// diagnostic build only: per wave {tile, column tile, band, y0, y1, interior
// columns, safe, cycles} of the last poisson_multi_kernel launch
extern "C" int cfd_march_stamps(long long* out, int n) {
  if (n > cfd::MARCH_STAMP_MAX * 8) n = cfd::MARCH_STAMP_MAX * 8;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(cfd::march_stamp_buf), (size_t)n * 8) == hipSuccess ? n : -1;
}
#endif

int cfd_set_field(cfd_solver* s, int field, const double* host, size_t count) {
  return guard([&] {
    if (!host) throw Error(CFD_E_ARG, "null host buffer");
    S_(s)->transfer(field, nullptr, host, count);
  });
}

int cfd_write_vtk(cfd_solver* s, const char* filename, double t) {
  return guard([&] {
    if (!filename) throw Error(CFD_E_ARG, "null filename");
    S_(s)->write_vtk(filename, t);
  });
}

int cfd_write_vtk_arrays(const cfd_params* p, const char* filename, double t, const double* uc, const double* vc,
                         const double* pr) {
  return guard([&] {
    if (!p || !filename || !uc || !vc || !pr) throw Error(CFD_E_ARG, "null argument");
    cfd::write_vtk_arrays(*p, filename, t, uc, vc, pr);
  });
}

int cfd_write_pvd(const char* filename, const char* const* files, const double* times, int n) {
  return guard([&] {
    if (!filename || n < 0 || (n > 0 && (!files || !times))) throw Error(CFD_E_ARG, "bad arguments");
    cfd::write_pvd(filename, files, times, n);
  });
}

int cfd_get_timing(cfd_solver* s, cfd_timing* out) {
  return guard([&] {
    if (!out) throw Error(CFD_E_ARG, "null output");
    Solver* v = S_(s);
    v->flush_step_time();
    v->flush_seq_count();
    *out = v->T;
  });
}
int cfd_reset_timing(cfd_solver* s) {
  return guard([&] {
    Solver* v = S_(s);
    v->flush_step_time();
    v->flush_seq_count();
    v->T = cfd_timing{};
  });
}
int cfd_synchronize(cfd_solver* s) { return guard([&] { HIPC(hipStreamSynchronize(S_(s)->st)); }); }
int cfd_set_tuning(cfd_solver* s, int knob, int value) { return guard([&] { S_(s)->set_tuning(knob, value); }); }

int cfd_owned_rows(const cfd_solver* s, int* first, int* last) {
  return guard([&] {
    if (!s || !s->impl || !first || !last) throw Error(CFD_E_ARG, "null argument");
    *first = s->impl->S.front().g.j0;
    *last = s->impl->S.back().g.j1;
  });
}

int cfd_comm_unique_id(unsigned char* id_out) {
  return guard([&] {
    if (!id_out) throw Error(CFD_E_ARG, "null id");
    cfd::comm_unique_id(id_out);
  });
}

void* cfd_comm_init(const unsigned char* id, int nranks, int rank, int device) {
  void* out = nullptr;
  guard([&] {
    if (!id) throw Error(CFD_E_ARG, "null id");
    out = cfd::comm_init(id, nranks, rank, device);
  });
  return out;
}

int cfd_comm_destroy(void* comm) { return guard([&] { cfd::comm_destroy(static_cast<cfd::Comm*>(comm)); }); }

int cfd_comm_info(void* comm, int* nranks, int* rank, int* transport) {
  return guard([&] {
    if (!nranks || !rank || !transport) throw Error(CFD_E_ARG, "null output");
    cfd::comm_info(static_cast<cfd::Comm*>(comm), nranks, rank, transport);
  });
}

int cfd_comm_exchange_check(void* comm, int peer, size_t count, long long* mismatches) {
  return guard([&] {
    if (!mismatches) throw Error(CFD_E_ARG, "null output");
    *mismatches = cfd::comm_exchange_check(static_cast<cfd::Comm*>(comm), peer, count);
  });
}

void* cfd_comm_loopback_hub(int nranks) {
  void* out = nullptr;
  guard([&] { out = cfd::loop_hub_create(nranks); });
  return out;
}

void* cfd_comm_init_loopback(void* hub, int rank, int device) {
  void* out = nullptr;
  guard([&] { out = cfd::comm_init_loopback(static_cast<cfd::LoopHub*>(hub), rank, device); });
  return out;
}

int cfd_comm_loopback_hub_destroy(void* hub) {
  return guard([&] { cfd::loop_hub_destroy(static_cast<cfd::LoopHub*>(hub)); });
}

}  // extern "C"
