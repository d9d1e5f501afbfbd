// p2v_version (include/p2v.h): the library version and the hash of the sources it was built from.
// P2V_SRC_HASH is srchash.py's digest of csrc/* and include/p2v.h, passed by the Makefile, which
// rebuilds this file whenever any of them changes; p2v.check_build() (bench.py, smoke()) recomputes
// it from the running tree and refuses a library built from other sources.
#include "../../include/p2v.h"

#ifndef P2V_SRC_HASH
#define P2V_SRC_HASH "unknown"
#endif

extern "C" const char* p2v_version(void) { return "p2v 0.1.0 (gfx950) src " P2V_SRC_HASH; }
