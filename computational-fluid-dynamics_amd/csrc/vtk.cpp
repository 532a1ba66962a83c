// vtk.cpp — frame output in the reference's legacy-VTK / PVD formats.
//
// VTKWriter::write_structured_grid: cavity-01.cpp:95-231 (cavity),
// channel-01.cpp:100-211 (channel), backwards_step-01.cpp:102-243 (masked
// step variant). The reference sets std::fixed + setprecision(6) on the file
// stream in the title line, so every number after it is printed as "%.6f";
// a few masked entries are string literals ("0.0"). write_paraview_collection:
// cavity-01.cpp:255-287.
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "internal.hpp"

namespace cfd {

bool host_is_fluid(const cfd_params& p, int j, int i) {
  if (i < 1 || i > p.nx || j < 1 || j > p.ny) return false;
  if (p.case_id != CFD_BACKSTEP) return true;
  return (i > p.step_i) || (j <= p.inlet_jmax);
}

namespace {

struct Out {
  std::string s;
  char buf[64];
  void num(double x) {
    int n = std::snprintf(buf, sizeof buf, "%.6f", x);
    s.append(buf, (size_t)n);
  }
  void lit(const char* t) { s.append(t); }
  void nl() { s.push_back('\n'); }
};

}  // namespace

void write_vtk_arrays(const cfd_params& p, const std::string& filename, double t, const double* uc,
                      const double* vc, const double* pr, const double* temp) {
  const int nx = p.nx, ny = p.ny, W = nx + 2;
  auto A = [W](const double* a, int j, int i) { return a[(size_t)j * W + i]; };
  const bool step = p.case_id == CFD_BACKSTEP;
  Out o;
  o.s.reserve((size_t)nx * ny * 80 + 1024);
  o.lit("# vtk DataFile Version 3.0\n");
  // Rayleigh-Benard frames: the cavity's layout and vorticity + a temperature field
  const bool rb = p.case_id == CFD_RAYLEIGH_BENARD;
  if (rb) o.lit("Rayleigh-Benard Convection Data - Time: ");
  else if (p.case_id == CFD_CAVITY) o.lit("Lid-Driven Cavity Flow Data - Time: ");
  else if (p.case_id == CFD_CHANNEL) o.lit("Channel Flow Data - Time: ");
  else o.lit("Backwards Step Flow Data - Time: ");
  o.num(t);
  o.nl();
  o.lit("ASCII\nDATASET STRUCTURED_POINTS\n");
  o.lit(("DIMENSIONS " + std::to_string(nx) + " " + std::to_string(ny) + " 1\n").c_str());
  const double dx = p.dx, dy = (p.case_id == CFD_CAVITY || rb) ? p.dx : p.dy;
  o.lit("ORIGIN ");
  o.num(dx * 0.5);
  o.lit(" ");
  o.num(dy * 0.5);
  o.lit(" 0.0\nSPACING ");
  o.num(dx);
  o.lit(" ");
  o.num(dy);
  o.lit(" 1.0\n");
  o.lit(("POINT_DATA " + std::to_string(nx * ny) + "\n").c_str());

  o.lit("SCALARS TimeValue double 1\nLOOKUP_TABLE default\n");
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) { o.num(t); o.nl(); }

  if (step) {
    o.lit("SCALARS FluidMask double 1\nLOOKUP_TABLE default\n");
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i) { o.num(host_is_fluid(p, j, i) ? 1.0 : 0.0); o.nl(); }
  }

  o.lit("VECTORS velocity double\n");
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) {
      if (step && !host_is_fluid(p, j, i)) { o.lit("0.0 0.0 0.0\n"); continue; }
      o.num(A(uc, j, i)); o.lit(" "); o.num(A(vc, j, i)); o.lit(" 0.0\n");
    }

  o.lit("SCALARS u_velocity double 1\nLOOKUP_TABLE default\n");
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) { o.num((!step || host_is_fluid(p, j, i)) ? A(uc, j, i) : 0.0); o.nl(); }
  o.lit("SCALARS v_velocity double 1\nLOOKUP_TABLE default\n");
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) { o.num((!step || host_is_fluid(p, j, i)) ? A(vc, j, i) : 0.0); o.nl(); }

  o.lit("SCALARS velocity_magnitude double 1\nLOOKUP_TABLE default\n");
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) {
      if (step && !host_is_fluid(p, j, i)) { o.lit("0.0\n"); continue; }
      const double a = A(uc, j, i), b = A(vc, j, i);
      o.num(std::sqrt(a * a + b * b));
      o.nl();
    }

  o.lit("SCALARS pressure double 1\nLOOKUP_TABLE default\n");
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) { o.num((!step || host_is_fluid(p, j, i)) ? A(pr, j, i) : 0.0); o.nl(); }

  if (rb && temp) {
    o.lit("SCALARS temperature double 1\nLOOKUP_TABLE default\n");
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i) { o.num(A(temp, j, i)); o.nl(); }
  }

  o.lit("SCALARS vorticity double 1\nLOOKUP_TABLE default\n");
  if (p.case_id == CFD_CAVITY || rb) {
    // cavity-01.cpp:187-224
    const int n_x = nx, n_y = ny;
    const double dx_inv = 1.0 / p.dx;
    for (int j = 1; j <= n_y; ++j)
      for (int i = 1; i <= n_x; ++i) {
        double w;
        if (i > 1 && i < n_x && j > 1 && j < n_y) {
          const double dvdx = (A(vc, j, i + 1) - A(vc, j, i - 1)) * dx_inv * 0.5;
          const double dudy = (A(uc, j + 1, i) - A(uc, j - 1, i)) * dx_inv * 0.5;
          w = dvdx - dudy;
        } else {
          double dvdx, dudy;
          if (i == 1) dvdx = (A(vc, j, i + 1) - A(vc, j, i)) * dx_inv;
          else if (i == n_x) dvdx = (A(vc, j, i) - A(vc, j, i - 1)) * dx_inv;
          else dvdx = (A(vc, j, i + 1) - A(vc, j, i - 1)) * dx_inv * 0.5;
          if (j == 1) dudy = (A(uc, j + 1, i) - A(uc, j, i)) * dx_inv;
          else if (j == n_y) dudy = (A(uc, j, i) - A(uc, j - 1, i)) * dx_inv;
          else dudy = (A(uc, j + 1, i) - A(uc, j - 1, i)) * dx_inv * 0.5;
          w = dvdx - dudy;
        }
        o.num(w);
        o.nl();
      }
  } else if (p.case_id == CFD_CHANNEL) {
    // channel-01.cpp:190-204
    const double idx = 1.0 / p.dx, idy = 1.0 / p.dy;
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i) {
        double dvdx, dudy;
        if (i == 1) dvdx = (A(vc, j, i + 1) - A(vc, j, i)) * idx;
        else if (i == nx) dvdx = (A(vc, j, i) - A(vc, j, i - 1)) * idx;
        else dvdx = 0.5 * (A(vc, j, i + 1) - A(vc, j, i - 1)) * idx;
        if (j == 1) dudy = (A(uc, j + 1, i) - A(uc, j, i)) * idy;
        else if (j == ny) dudy = (A(uc, j, i) - A(uc, j - 1, i)) * idy;
        else dudy = 0.5 * (A(uc, j + 1, i) - A(uc, j - 1, i)) * idy;
        o.num(dvdx - dudy);
        o.nl();
      }
  } else {
    // backwards_step-01.cpp:210-236
    const double idx = 1.0 / p.dx, idy = 1.0 / p.dy;
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i) {
        if (!host_is_fluid(p, j, i)) { o.lit("0.0\n"); continue; }
        bool ok = !(i == 1 || i == nx || j == 1 || j == ny);
        if (ok && (!host_is_fluid(p, j, i - 1) || !host_is_fluid(p, j, i + 1) || !host_is_fluid(p, j - 1, i) ||
                   !host_is_fluid(p, j + 1, i)))
          ok = false;
        if (ok) {
          const double dvdx = 0.5 * (A(vc, j, i + 1) - A(vc, j, i - 1)) * idx;
          const double dudy = 0.5 * (A(uc, j + 1, i) - A(uc, j - 1, i)) * idy;
          o.num(dvdx - dudy);
          o.nl();
        } else {
          o.lit("0.0\n");
        }
      }
  }

  FILE* f = std::fopen(filename.c_str(), "wb");
  if (!f) throw Error(CFD_E_IO, "Cannot open file: " + filename);
  const size_t w = std::fwrite(o.s.data(), 1, o.s.size(), f);
  const int rc = std::fclose(f);
  if (w != o.s.size() || rc != 0) throw Error(CFD_E_IO, "Error writing to file: " + filename);
}

void write_pvd(const std::string& filename, const char* const* files, const double* times, int n) {
  std::string s = "<?xml version=\"1.0\"?>\n"
                  "<VTKFile type=\"Collection\" version=\"0.1\" byte_order=\"LittleEndian\">\n"
                  "  <Collection>\n";
  char buf[64];
  for (int k = 0; k < n; ++k) {
    std::snprintf(buf, sizeof buf, "%.6f", times[k]);
    s += "    <DataSet timestep=\"";
    s += buf;
    s += "\" group=\"\" part=\"0\" file=\"";
    s += files[k];
    s += "\"/>\n";
  }
  s += "  </Collection>\n</VTKFile>\n";
  FILE* f = std::fopen(filename.c_str(), "wb");
  if (!f) throw Error(CFD_E_IO, "Cannot open collection file: " + filename);
  const size_t w = std::fwrite(s.data(), 1, s.size(), f);
  const int rc = std::fclose(f);
  if (w != s.size() || rc != 0) throw Error(CFD_E_IO, "Error writing collection file: " + filename);
}

}  // namespace cfd
