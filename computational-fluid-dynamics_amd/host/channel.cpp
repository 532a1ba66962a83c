// channel.cpp — drop-in for the reference's ./channel binary (see driver.hpp).
#include "driver.hpp"

int main(int argc, char** argv) { return host::run_case(CFD_CHANNEL, argc, argv); }
