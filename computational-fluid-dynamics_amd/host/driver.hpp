// driver.hpp — the drop-in host program shared by bin/cavity, bin/channel and
// bin/backwards_step: the reference's main() + run() loop (cavity-01.cpp:374-411,
// 781-796; channel-01.cpp:360-396; backwards_step-01.cpp:404-440) over the
// C-ABI of libcfd_amd.so, with the README's CLI (--Re/--Nx/--Ny/--dt).
#pragma once

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "cfd_amd.h"

namespace host {

constexpr char RESET[] = "\033[0m";
constexpr char RED[] = "\033[31m";
constexpr char GREEN[] = "\033[32m";
constexpr char YELLOW[] = "\033[33m";
constexpr char BLUE[] = "\033[34m";
constexpr char CYAN[] = "\033[36m";

struct Options {
  double re = 0, dt = 0, final_time = 0, ra = 0, pr = 0;
  int nx = 0, ny = 0, steps = -1, max_iters = 0, save = 0, print = 0, device = 0, strips = 1, check_every = 1;
  bool vtk = true;
  bool red_black = false;
  bool exact_given = false;
  std::string outdir = "vtk_output";
};

inline void usage(const char* prog) {
  std::cerr << "usage: " << prog
            << " [--Re R | --Ra RA --Pr PR] [--Nx N] [--Ny N] [--dt DT] [--final-time T] [--steps K] [--max-iters N]\n"
               "       [--save-interval N] [--print-interval N] [--output-dir DIR] [--no-vtk]\n"
               "       [--device D] [--strips S] [--check-every C] [--red-black] [--exact]\n"
               "  default: the reference's lexicographic SOR order (bit-identical output; strips allowed)\n"
               "  --red-black: red-black SOR order (the multi-GPU order; the same answer where the\n"
               "               solve converges, a different iterate where it hits the sweep cap)\n"
               "  --exact: the reference's order (the default; kept for older scripts)\n";
}

inline Options parse(int argc, char** argv) {
  Options o;
  for (int k = 1; k < argc; ++k) {
    std::string a = argv[k];
    auto next = [&]() -> const char* {
      if (k + 1 >= argc) {
        usage(argv[0]);
        std::exit(2);
      }
      return argv[++k];
    };
    if (a == "--Re") o.re = std::atof(next());
    else if (a == "--Ra") o.ra = std::atof(next());
    else if (a == "--Pr") o.pr = std::atof(next());
    else if (a == "--Nx") o.nx = std::atoi(next());
    else if (a == "--Ny") o.ny = std::atoi(next());
    else if (a == "--dt") o.dt = std::atof(next());
    else if (a == "--final-time") o.final_time = std::atof(next());
    else if (a == "--steps") o.steps = std::atoi(next());
    else if (a == "--max-iters") o.max_iters = std::atoi(next());
    else if (a == "--save-interval") o.save = std::atoi(next());
    else if (a == "--print-interval") o.print = std::atoi(next());
    else if (a == "--output-dir") o.outdir = next();
    else if (a == "--no-vtk") o.vtk = false;
    else if (a == "--exact") o.red_black = false, o.exact_given = true;
    else if (a == "--red-black") o.red_black = true;
    else if (a == "--device") o.device = std::atoi(next());
    else if (a == "--strips") o.strips = std::atoi(next());
    else if (a == "--check-every") o.check_every = std::atoi(next());
    else if (a == "-h" || a == "--help") {
      usage(argv[0]);
      std::exit(0);
    } else {
      std::cerr << "unknown argument " << a << "\n";
      usage(argv[0]);
      std::exit(2);
    }
  }
  return o;
}

inline void die(const char* what) {
  std::cerr << RED << "Error: " << what << ": " << cfd_last_error() << RESET << "\n";
  std::exit(1);
}

inline std::string frame_name(const std::string& base, int step) {
  std::ostringstream oss;
  oss << base << "_" << std::setfill('0') << std::setw(6) << step << ".vtk";
  return oss.str();
}

inline int run_case(int case_id, int argc, char** argv) {
  const Options o = parse(argc, argv);
  cfd_params p;
  const bool rb = case_id == CFD_RAYLEIGH_BENARD;
  if (rb) {
    if (cfd_params_init_rb(o.ra, o.pr, o.nx, o.ny, o.dt, &p) != CFD_OK) die("parameters");
  } else if (cfd_params_init(case_id, o.re, o.nx, o.ny, o.dt, &p) != CFD_OK) {
    die("parameters");
  }
  if (o.final_time > 0) {
    p.final_time = o.final_time;
    p.total_steps = (int)(p.final_time / p.dt);
  }
  if (o.max_iters > 0) p.max_iters = o.max_iters;
  if (o.save > 0) p.save_interval = o.save;
  if (o.print > 0) p.print_interval = o.print;
  p.check_every = o.check_every;
  // cfd_params_init's default is the reference's order; Rayleigh-Benard (no
  // reference solver) keeps red-black unless asked
  if (o.red_black) p.ordering = CFD_ORDER_RB;
  else if (!rb || o.exact_given) p.ordering = CFD_ORDER_LEX;
  const int total = o.steps >= 0 ? o.steps : p.total_steps;
  const char* base = case_id == CFD_CAVITY    ? "cavity_flow"
                     : case_id == CFD_CHANNEL ? "channel_flow"
                     : rb                     ? "rayleigh_benard"
                                              : "backwards_step";
  const std::string coll = std::string(base) + (case_id == CFD_BACKSTEP ? "_animation.pvd" : "_animation.pvd");

  if (case_id == CFD_BACKSTEP) {
    // backwards_step-01.cpp:495-531 (printed before the stream is switched to fixed)
    const long long fluid = (long long)p.nx * p.ny - (long long)p.step_i * (p.ny - p.inlet_jmax);
    std::cout << CYAN << "Setting up backwards step geometry:\n"
              << "  Step location: x = " << p.step_x << " (i = " << p.step_i << ")\n"
              << "  Inlet height: " << p.h_inlet << " (j = 1 to " << p.inlet_jmax << ")\n"
              << "  Total height: " << p.height << " (j = 1 to " << p.ny << ")\n"
              << RESET;
    std::cout << BLUE << "Geometry setup complete. Fluid cells: " << fluid << "/" << (p.nx * p.ny) << RESET << "\n";
  }
  if (o.vtk) {
    std::filesystem::create_directories(o.outdir);
    std::cout << BLUE << "Created output directory: " << o.outdir << RESET << "\n";
  }
  std::cout << std::fixed << std::setprecision(6);
  std::cout << CYAN;
  if (rb) {
    std::cout << "=== Rayleigh-Benard Convection Simulation ===\n"
              << "Domain: " << p.length << "x" << p.height << "\n"
              << "Grid: " << p.nx << "x" << p.ny << " (spacing=" << p.dx << ")\n"
              << "Rayleigh=" << p.ra << ", Prandtl=" << p.pr << ", thermal diffusivity=" << p.kappa << "\n";
  } else if (case_id == CFD_CAVITY) {
    std::cout << "=== Lid-Driven Cavity Flow Simulation ===\n"
              << "Domain: " << p.length << "x" << p.height << "\n"
              << "Grid: " << p.nx << "x" << p.ny << " (spacing=" << p.dx << ")\n";
  } else if (case_id == CFD_CHANNEL) {
    std::cout << "=== Channel Flow Simulation ===\n"
              << "Domain: " << p.length << "x" << p.height << "\n"
              << "Grid: " << p.nx << "x" << p.ny << " (dx=" << p.dx << ", dy=" << p.dy << ")\n";
  } else {
    std::cout << "=== Backwards Step Flow Simulation ===\n"
              << "Domain: " << p.length << "x" << p.height << "\n"
              << "Step: height=" << (p.height - p.h_inlet) << ", location=" << p.step_x << "\n"
              << "Grid: " << p.nx << "x" << p.ny << " (dx=" << p.dx << ", dy=" << p.dy << ")\n";
  }
  std::cout << "Time: dt=" << p.dt << ", steps=" << p.total_steps << ", final_time=" << p.final_time << "\n"
            << "Reynolds=" << p.re << ", kinematic viscosity=" << p.nu << ", CFL=" << p.cfl << "\n"
            << "Relaxation factor=" << p.omega << "\n"
            << "VTK export interval=" << p.save_interval << " steps\n"
            << "==========================================\n"
            << RESET << "\n";

  cfd_solver* s = cfd_create(&p, o.device, o.strips);
  if (!s) die("cfd_create");
  std::vector<std::string> files;
  std::vector<double> times;
  auto exportf = [&](int k, double t) {
    if (!o.vtk) return;
    const std::string fn = frame_name(base, k);
    if (cfd_write_vtk(s, (o.outdir + "/" + fn).c_str(), t) != CFD_OK) {
      std::cerr << RED << "Error exporting VTK data: " << cfd_last_error() << RESET << "\n";
      return;
    }
    files.push_back(fn);
    times.push_back(t);
    if (k % p.print_interval == 0 || k == 0) std::cout << BLUE << "Exported VTK file: " << fn << RESET << "\n";
  };

  // Nusselt number at the hot wall from the bottom interior row of T
  std::vector<double> tfield;
  auto nusselt = [&]() {
    int rows = 0, cols = 0;
    if (cfd_field_shape(s, CFD_FIELD_T, &rows, &cols) != CFD_OK) die("field_shape");
    tfield.resize((size_t)rows * cols);
    if (cfd_get_field(s, CFD_FIELD_T, tfield.data(), tfield.size()) != CFD_OK) die("get_field");
    double q = 0;
    for (int i = 1; i <= p.nx; ++i) q += (p.t_hot - tfield[(size_t)cols + i]) / (0.5 * p.dy);
    return q / p.nx / (p.t_hot - p.t_cold);
  };
  if (case_id == CFD_CAVITY || rb) {
    std::cout << GREEN << "Starting simulation...\n" << RESET;
    if (cfd_apply_bc(s) != CFD_OK) die("applyBoundaryConditions");
    exportf(0, 0.0);
  } else {
    exportf(0, 0.0);
    std::cout << GREEN << (case_id == CFD_CHANNEL ? "Starting simulation...\n" : "Starting backwards step simulation...\n")
              << RESET;
  }
  for (int k = 1; k <= total; ++k) {
    const double t = k * p.dt;
    cfd_step_info info;
    if (cfd_step(s, &info) != CFD_OK) die("timestep");
    if (info.sor_iterations >= p.max_iters) {
      if (case_id == CFD_CAVITY || rb)
        std::cerr << "Warning: SOR solver did not converge in " << p.max_iters
                  << " iterations. Final residual: " << info.residual << "\n";
      else
        std::cerr << YELLOW << "Warning: PPE SOR hit max iterations, max_res=" << info.residual << RESET << "\n";
    }
    if (k % p.print_interval == 0 || k == total) {
      cfd_stats st;
      if (cfd_compute_stats(s, &st) != CFD_OK) die("logStatistics");
      if (rb)
        std::cout << "Step " << std::setw(6) << k << "/" << p.total_steps << " | t=" << std::fixed << std::setprecision(2)
                  << std::setw(6) << t << " | max(div)=" << std::setprecision(2) << std::scientific << std::setw(10)
                  << st.max_divergence << " | avg_KE=" << std::fixed << std::setprecision(6) << std::setw(10)
                  << st.avg_kinetic_energy << " | Nu=" << std::setprecision(4) << nusselt()
                  << " | SOR_iters=" << std::setw(4) << info.sor_iterations << "\n";
      else if (case_id == CFD_CAVITY)
        std::cout << "Step " << std::setw(6) << k << "/" << p.total_steps << " | t=" << std::fixed << std::setprecision(2)
                  << std::setw(6) << t << " | max(div)=" << std::setprecision(2) << std::scientific << std::setw(10)
                  << st.max_divergence << " | avg_KE=" << std::fixed << std::setprecision(6) << std::setw(10)
                  << st.avg_kinetic_energy << " | SOR_iters=" << std::setw(4) << info.sor_iterations << "\n";
      else
        std::cout << "Step " << std::setw(6) << k << "/" << p.total_steps << " | t=" << std::fixed << std::setprecision(3)
                  << std::setw(8) << t << " | max(div)=" << std::scientific << std::setprecision(2) << std::setw(10)
                  << st.max_divergence << " | avg_KE=" << std::fixed << std::setprecision(6) << std::setw(10)
                  << st.avg_kinetic_energy << " | PPE iters=" << std::setw(4) << info.sor_iterations
                  << " | res=" << std::scientific << std::setprecision(2) << std::setw(10) << info.residual << "\n";
      std::cout.flush();  // (progress lines reach a pipe as they are printed)
    }
    if (k % p.save_interval == 0 || k == total) exportf(k, t);
  }
  if (o.vtk) {
    std::vector<const char*> names;
    for (auto& f : files) names.push_back(f.c_str());
    if (cfd_write_pvd((o.outdir + "/" + coll).c_str(), names.data(), times.data(), (int)names.size()) != CFD_OK)
      std::cerr << RED << "Error creating ParaView collection: " << cfd_last_error() << RESET << "\n";
    else
      std::cout << CYAN << "Created ParaView collection file: " << coll << RESET << "\n";
  }
  cfd_destroy(s);
  std::cout << GREEN << "Simulation completed successfully!\n";
  if (o.vtk)
    std::cout << "VTK files saved in directory: " << o.outdir << "\n"
              << "Open '" << o.outdir << "/" << coll << "' in ParaView for animation\n";
  std::cout << RESET;
  return 0;
}

}  // namespace host
