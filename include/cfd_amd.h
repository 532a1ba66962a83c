/*
 * include/cfd_amd.h — C-ABI of libcfd_amd.so, the MI355X-native projection
 * solver (lid-driven cavity, channel, backwards-facing step).
 *
 * The reference has no FFI: each case is one C++ class driven by main()
 * (cavity-01.cpp:306-775, channel-01.cpp:284-770, backwards_step-01.cpp:316-1062).
 * The entry points below are that class's per-timestep methods, exported with
 * plain pointers and sizes so a host in any language can bind them. Each
 * declaration names the reference method it replaces. All functions return
 * 0 on success and a negative CFD_E_* code on failure; cfd_last_error()
 * then describes the failure. No function falls back to a CPU path: if no
 * usable gfx950 device is present, cfd_create fails.
 */
#ifndef CFD_AMD_H
#define CFD_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CFD_AMD_ABI_VERSION 13

/* CFD_RAYLEIGH_BENARD (BASELINE configs[4]) has no solver in the reference
 * tree (only figures): it is the cavity's projection step with a resting lid
 * plus a Boussinesq temperature field; see DESIGN.md §5c ("parity unpinned"). */
enum cfd_case { CFD_CAVITY = 0, CFD_CHANNEL = 1, CFD_BACKSTEP = 2, CFD_RAYLEIGH_BENARD = 3 };

/* Fields, named after the reference members (cavity-01.cpp:336-344). */
enum cfd_field {
  CFD_FIELD_P = 0,    /* pressure            (ny+2) x (nx+2) */
  CFD_FIELD_SRC = 1,  /* source_term         (ny+2) x (nx+2) */
  CFD_FIELD_US = 3,   /* u_tentative         (ny+2) x (nx+1) */
  CFD_FIELD_VS = 4,   /* v_tentative         (ny+1) x (nx+2) */
  CFD_FIELD_U = 5,    /* u_corrected         (ny+2) x (nx+1) */
  CFD_FIELD_V = 6,    /* v_corrected         (ny+1) x (nx+2) */
  CFD_FIELD_UC = 7,   /* u_center            (ny+2) x (nx+2) */
  CFD_FIELD_VC = 8,   /* v_center            (ny+2) x (nx+2) */
  CFD_FIELD_T = 9     /* temperature (Rayleigh-Benard only) (ny+2) x (nx+2) */
};

enum {
  CFD_OK = 0,
  CFD_E_ARG = -1,      /* invalid argument */
  CFD_E_DEVICE = -2,   /* HIP runtime / device failure */
  CFD_E_COMM = -3,     /* RCCL failure */
  CFD_E_STATE = -4,    /* call not valid in the current state */
  CFD_E_IO = -5        /* file output failure */
};

/*
 * Solver parameters: the reference's derived constants (cavity-01.cpp:322-327,
 * channel-01.cpp:302-308, backwards_step-01.cpp:337-352). Hosts derive them
 * from the CLI with cfd_params_init(); all fields may then be overridden.
 */
typedef struct cfd_params {
  int case_id;          /* enum cfd_case */
  int nx, ny;           /* global interior cells */
  double length, height;
  double re, u_ref, rho, cfl, final_time;
  double dx, dy, nu, dt, omega;
  double tol_factor, abs_tol;
  int max_iters;        /* MAX_SOR_ITERS */
  int total_steps;
  int print_interval, save_interval;
  double h_inlet, step_x;  /* backwards step geometry */
  int step_i, inlet_jmax;  /* derived step indices (backwards_step-01.cpp:386, 493) */
  int check_every;      /* residual test every N SOR iterations (1 = reference; red-black orders:
                           the reference order tests every iteration) */
  int chunk;            /* SOR launches enqueued between host polls (0 = auto) */
  int ordering;         /* CFD_ORDER_LEX (cfd_params_init's default: the reference's own sweep order,
                           bit-identical to the reference binaries - every case at any size, on strips of
                           one device and on ranks (ABI 12): the same bits at every strip / rank count) or
                           CFD_ORDER_RB (red-black: faster where the reference's solve converges, and its
                           rank launches overlap the halo exchange with the interior rows) */
  int sweeps_per_launch; /* SOR iterations fused into one kernel launch, bit-identical for every value:
                           0 = auto: red-black with the proof-mode test 4 (the backwards step on strips or
                           ranks: 3), red-black with exact residuals 3 (cavity) / 2 (channel, step);
                           lexicographic order 4 (3 on strips); 1, 2; 3 (red-black: cavity only, every
                           launch 3); 4 (red-black with the proof test, or the lexicographic order: the
                           auto plan, stated); 5 (lexicographic cavity on one strip). Ignored by the
                           one-workgroup solves (small_solve) */
  /* Rayleigh-Benard (case 3), free-fall units: H = 1, U = sqrt(g beta dT H),
   * nu = sqrt(Pr/Ra), kappa = 1/sqrt(Ra Pr); hot bottom wall t_hot, cold top
   * wall t_cold, adiabatic side walls; buoyancy (T - t_ref) on v. */
  double ra, pr, kappa, buoyancy, t_hot, t_cold, t_ref;
  double t_perturb;     /* initial T = conduction profile + t_perturb*sin(pi y)cos(pi x/L) */
  /* Solve-path switches (enum cfd_switch; cfd_params_init sets CFD_AUTO). None of them changes a
   * result bit (iteration counts, residuals, fields); they choose how the same solve runs. */
  int proof_test;       /* red-black launches: proof-mode convergence test where it applies -
                           every case (AUTO / ON); OFF: the max-norm residual in every tested sweep */
  int small_solve;      /* one strip, no ranks, p fits the LDS: the whole solve in one workgroup - red-black
                           (small.hpp) or the reference's order (smlex.hip) (AUTO / ON); OFF: the
                           multi-launch solve */
  int overlap;          /* ranks with >= 48 rows: halo exchange overlapped with the interior rows
                           (AUTO / ON); OFF: exchange in front of each launch */
} cfd_params;

enum cfd_switch { CFD_AUTO = 0, CFD_ON = 1, CFD_OFF = 2 };

enum cfd_ordering { CFD_ORDER_RB = 0, CFD_ORDER_LEX = 1 };

typedef struct cfd_solver cfd_solver;

typedef struct cfd_step_info {
  int sor_iterations;   /* SolverResult.first  (cavity-01.cpp:689) */
  double residual;      /* SolverResult.second (max-norm PPE residual) */
} cfd_step_info;

typedef struct cfd_stats {
  double max_divergence;      /* logStatistics, cavity-01.cpp:757-764 */
  double avg_kinetic_energy;  /* logStatistics, cavity-01.cpp:750-766 */
} cfd_stats;

typedef struct cfd_timing {
  double poisson_ms;          /* device time inside SOR launches (HIP events) */
  long long poisson_launches; /* SOR kernel launches that did work */
  long long poisson_cell_updates; /* interior cells x active iterations (this rank) */
  double step_ms;             /* device time of whole timesteps */
  long long steps;
  long long poisson_sweeps;   /* SOR iterations executed by those launches (up to 4 per fused launch) */
  long long poisson_overlapped; /* pair launches split into interior + halo-overlapped boundary rows (ranks) */
  double poisson_steady_ms;   /* lexicographic order: device time of the launches with every cell active */
  long long poisson_steady_launches; /* (the ramps at the start / end of a solve excluded) */
  long long proof_fallbacks;  /* red-black cavity: solves whose proof-mode convergence test left an
                                 iteration open, finished with exact residuals */
  int sor_kernel;             /* enum cfd_sor_kernel: the SOR kernel family of the last solve (ABI 8) */
  long long resident_timeouts; /* resident whole-solve launches whose tiles' waits timed out (never expected:
                                  the plan checks co-residency); the exact launches took those solves (ABI 12) */
  long long seqsum_chunks;        /* reference order: chunks of SQ_CH terms the sequential sums (source mean,
                                     kinetic energy) were cut into (ABI 13) */
  long long seqsum_serial_chunks; /* of those, the chunks that ran as the plain chain of adds (the first terms
                                     from zero, binade crossings, ties); the rest were exact integer sums (ABI 13) */
} cfd_timing;

/* Which SOR kernel family ran a solve (cfd_timing.sor_kernel); every one gives the same bits for
 * the same ordering. */
enum cfd_sor_kernel {
  CFD_SOR_NONE = 0,
  CFD_SOR_MARCH = 1,  /* red-black wave-march launches (kernels.hpp), any size, strips and ranks */
  CFD_SOR_TILE = 2,   /* red-black LDS-tile launches (tile.hpp): one strip of up to ~4 M cells */
  CFD_SOR_SMALL = 3,  /* red-black whole solve in one workgroup (small.hpp): reference-sized grids */
  CFD_SOR_LEXW = 4,   /* reference order, multi-block march (lexw.hpp) */
  CFD_SOR_LEX = 5,    /* reference order, one workgroup, global memory (poisson_lex_kernel: step geometries
                         the other reference-order kernels do not take) */
  CFD_SOR_SMLEX = 6,  /* reference order, whole solve in one workgroup, p in LDS (smlex.hip): reference-sized
                         grids (ABI 9) */
  CFD_SOR_RESIDENT = 7 /* whole solve in one persistent launch, every tile of p in registers (resident.hpp):
                          the cavity and the channel, both orders, one strip of up to ~2 M cells, no ranks
                          (ABI 11) */
};

/* Library / ABI info. */
int cfd_abi_version(void);
const char* cfd_last_error(void);

/* Reference constants for a case with CLI overrides (<=0 / NULL keeps the
 * reference value): the constructor initialisers of the reference classes
 * (cavity-01.cpp:355-364, channel-01.cpp:336-345, backwards_step-01.cpp:377-388). */
int cfd_params_init(int case_id, double re, int nx, int ny, double dt, cfd_params* out);

/* Rayleigh-Benard parameters (no reference counterpart; BASELINE configs[4]):
 * Ra, Pr, grid (aspect L = nx/ny, H = 1, dx = dy), dt (<= 0: CFL-derived).
 * cfd_params_init(CFD_RAYLEIGH_BENARD, ra, nx, ny, dt, out) = this with Pr 0.71. */
int cfd_params_init_rb(double ra, double pr, int nx, int ny, double dt, cfd_params* out);

/* Construct a solver: CavitySolver()/ChannelSolver()/BackwardsStepSolver()
 * (cavity-01.cpp:355, channel-01.cpp:336, backwards_step-01.cpp:377) —
 * allocateFields + setupGeometry + the initial applyBoundaryConditions of the
 * open cases. The grid is split into `n_strips` row strips on this device
 * (1 = one domain); strips exchange halo rows after every stage. */
cfd_solver* cfd_create(const cfd_params* p, int device, int n_strips);

/* Multi-process construction: this rank owns interior rows
 * [row_begin, row_end] (1-based, inclusive) of the global grid; neighbour
 * halos travel over RCCL (see cfd_comm_*). Both orderings (ABI 12: the
 * reference's order too - halo rows before every launch, the stop rule's
 * exceedance bits OR-ed over the ranks, the sequential sums chained rank to
 * rank: bit-identical to one device). */
cfd_solver* cfd_create_rank(const cfd_params* p, int device, int row_begin, int row_end, void* comm);
int cfd_destroy(cfd_solver* s);

/* Per-timestep methods. */
int cfd_apply_bc(cfd_solver* s);                  /* applyBoundaryConditions   cavity-01.cpp:523 / channel-01.cpp:509 */
int cfd_apply_tentative_bc(cfd_solver* s);        /* applyVelocityBC(u*,v*)    channel-01.cpp:369 */
int cfd_compute_tentative(cfd_solver* s);         /* computeTentativeVelocities cavity-01.cpp:548 */
/* Rayleigh-Benard only: temperature ghost cells, buoyancy added to v* and one
 * explicit advection-diffusion update of T (fused kernel); cfd_step runs it
 * between cfd_compute_tentative and cfd_build_source. */
int cfd_advance_temperature(cfd_solver* s);
int cfd_build_source(cfd_solver* s);              /* source term (+ mean removal) cavity-01.cpp:622 / channel-01.cpp:608 */
int cfd_solve_pressure(cfd_solver* s, cfd_step_info* out); /* solverPressurePoisson cavity-01.cpp:609 */
int cfd_apply_correction(cfd_solver* s);          /* applyPressureCorrection   cavity-01.cpp:695 */
int cfd_step(cfd_solver* s, cfd_step_info* out);  /* one iteration of run()'s loop, cavity-01.cpp:387-390 */
int cfd_run_steps(cfd_solver* s, int n_steps, cfd_step_info* last); /* n loop iterations, no logging */

/* interpolateToCellCenters + logStatistics reductions (cavity-01.cpp:717, 741). */
int cfd_compute_stats(cfd_solver* s, cfd_stats* out);

/* Field transfer in the reference's array shapes (see enum cfd_field), as
 * dense row-major doubles: rows x cols with rows/cols from cfd_field_shape.
 * For a rank solver only the rank's owned rows are transferred. */
int cfd_field_shape(const cfd_solver* s, int field, int* rows, int* cols);
int cfd_get_field(cfd_solver* s, int field, double* host, size_t count);
int cfd_set_field(cfd_solver* s, int field, const double* host, size_t count);

/* VTKWriter::write_structured_grid (cavity-01.cpp:95-231; masked variant
 * backwards_step-01.cpp:102-243) and write_paraview_collection
 * (cavity-01.cpp:255-287). */
int cfd_write_vtk(cfd_solver* s, const char* filename, double time_value);
int cfd_write_pvd(const char* filename, const char* const* vtk_files, const double* times, int n);

/* Host-only VTK formatting of given cell-centre / pressure arrays, each a
 * dense (ny+2) x (nx+2) row-major array in the reference's indexing. */
int cfd_write_vtk_arrays(const cfd_params* p, const char* filename, double time_value, const double* u_center,
                         const double* v_center, const double* pressure);

/* Interior rows [first, last] (global, 1-based) this solver owns. */
int cfd_owned_rows(const cfd_solver* s, int* first, int* last);

/* Launch-planning knobs (performance only: every value gives the same bits).
 * Defaults are the values measured best on MI355X. */
enum cfd_tuning {
  CFD_TUNE_PAIR_WPS = 0,      /* waves per SIMD the fused red-black launch is planned for (1..4) */
  CFD_TUNE_WAVE_WPS = 1,      /* the same for the one-sweep launch */
  CFD_TUNE_LEXW_WAVES = 2,    /* tiles per lexicographic-order launch (>= 64) */
  CFD_TUNE_LEXW_EDGE_PCT = 3, /* wall-tile band length, % of the interior band (10..100; default 75 up to
                                 2048 rows, 100 above) */
  CFD_TUNE_PAIR_EDGE_PCT = 4, /* boundary-column band length of red-black launches, % (10..100) */
  CFD_TUNE_MARCH_MIN_TH = 5,  /* minimum rows per band of a march launch (>= 1; default 16 for the channel
                                 and for the reference order, 24 for the red-black cavity / step) */
  CFD_TUNE_TENT_TH = 6,       /* rows per band of the predictor's march (>= 4) */
  CFD_TUNE_LEXW_RAMP_PCT = 7, /* lexicographic ramp launches: band height floor, % of the steady plan's (0..100) */
  CFD_TUNE_TILE_ROUNDS = 8,   /* red-black, one strip: LDS-tile launches when the grid fits this many
                                 resident rounds of tiles (one per CU; 0: never, the march launches;
                                 default 1 for the cavity, 0 for the open cases) */
  CFD_TUNE_MARCH_ORDER = 9,   /* red-black march launches: 0 = the column tiles of a band on consecutive waves
                                 (default), 1 = the bands of a column tile (ABI 9) */
  CFD_TUNE_LEXW_LEFT = 10,    /* reference-order backwards step: 1 = the column tiles left of the step's column end
                                 at the block's bottom row and march as a channel below it (default), 0 = the
                                 per-cell masked march over every row that reaches the block (ABI 10) */
  CFD_TUNE_RESIDENT = 11,     /* the cavity and the channel, one strip, no ranks, both orders (red-black: with the
                                 proof-mode test; the reference order: sampled exceedance bits, an iteration they
                                 leave open finished by the multi-block march): 1 = the whole solve as one
                                 persistent register-resident launch where the grid fits one tile per CU and every
                                 tile can be resident at once (default: cavity 1024^2 2.2 us per sweep against the
                                 LDS tiles' 5.2), 0 = never (ABI 11) */
  CFD_TUNE_LEXW_UPDOWN = 12   /* reference order, wholly active interior tiles: 1 = every other band marches up
                                 (no residuals there; neighbouring bands read their shared halo rows at the same
                                 time), 0 = every band marches down (ABI 12) */
};
int cfd_set_tuning(cfd_solver* s, int knob, int value);
/* The default a solver created from these parameters starts with (host only, no
 * device needed; ABI 9). The waves-per-SIMD knobs (PAIR_WPS, WAVE_WPS,
 * LEXW_WAVES) come from the device's occupancy: CFD_E_STATE. */
int cfd_tuning_default(const cfd_params* p, int knob, int* value);

/* Timing collected with HIP events on the solver's stream. */
int cfd_get_timing(cfd_solver* s, cfd_timing* out);
int cfd_reset_timing(cfd_solver* s);
int cfd_synchronize(cfd_solver* s);

/* RCCL bootstrap for multi-process strip decomposition: rank 0 creates an id
 * (opaque bytes, CFD_COMM_ID_BYTES), every rank passes it to cfd_comm_init. */
#define CFD_COMM_ID_BYTES 128
int cfd_comm_unique_id(unsigned char* id_out);
void* cfd_comm_init(const unsigned char* id, int nranks, int rank, int device);
int cfd_comm_destroy(void* comm);
/* What the transport itself reports: for RCCL, ncclCommCount / ncclCommUserRank
 * (so a host can show that RCCL saw every rank); transport 0 = RCCL, 1 = loopback. */
int cfd_comm_info(void* comm, int* nranks, int* rank, int* transport);

/* Transport check (ABI 10): one halo exchange through the solver's own send / recv group
 * (comm.hip comm_halo_exchange, as Solver::exchange issues it) with `peer` as both neighbours, on
 * device buffers of `count` doubles holding a (rank, side, index) pattern; *mismatches = doubles
 * received that differ from the peer's pattern. peer = the caller's rank exercises RCCL's send /
 * recv to self, which a one-GPU host can run. */
int cfd_comm_exchange_check(void* comm, int peer, size_t count, long long* mismatches);

/* In-process transport with the same semantics, for ranks that share one
 * device and run in separate host threads of one process (RCCL refuses two
 * ranks on one GPU): exercises the rank code path without RCCL. */
void* cfd_comm_loopback_hub(int nranks);
void* cfd_comm_init_loopback(void* hub, int rank, int device);
int cfd_comm_loopback_hub_destroy(void* hub);

#ifdef __cplusplus
}
#endif
#endif
