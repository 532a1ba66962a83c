// rayleigh_benard.cpp — Rayleigh-Benard convection (BASELINE configs[4]; the
// reference has figures of it but no solver) with the drop-in binaries' CLI
// plus --Ra/--Pr (see driver.hpp).
#include "driver.hpp"

int main(int argc, char** argv) { return host::run_case(CFD_RAYLEIGH_BENARD, argc, argv); }
