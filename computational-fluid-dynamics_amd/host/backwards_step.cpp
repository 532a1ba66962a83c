// backwards_step.cpp — drop-in for the reference's ./backwards_step binary (see driver.hpp).
#include "driver.hpp"

int main(int argc, char** argv) { return host::run_case(CFD_BACKSTEP, argc, argv); }
