// The C-ABI version the library was built for (include/regnn_hip.h, "ABI version"). Kept in its
// own translation unit so that bumping it leaves the kernel sources' content hashes (PMC
// summaries, build.kernel_hash) unchanged.
#include "regnn_common.h"

extern "C" int regnn_abi_version(void) { return 46; }
