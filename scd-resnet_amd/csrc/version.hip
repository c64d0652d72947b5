// Library identity: scd_version() = "libscdhip <abi> gfx950 <build id>", the build id being a hash of the sources the
// library was built from (Makefile BUILD_ID; a variant build appends "+<name>").  bench.py compares it with the
// identity stamped into a PMC summary before attributing that summary's bytes to this library's kernels.
#include "scd_common.h"

#ifndef SCD_BUILD_ID
#define SCD_BUILD_ID "unknown"
#endif

extern "C" const char* scd_version(void) { return "libscdhip 0.2 gfx950 " SCD_BUILD_ID; }
