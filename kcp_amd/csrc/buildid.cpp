// The build ID: kcp_amd/buildinfo.py's SHA-256 over the contents of every source, header, map and build
// script of this library, passed in by kcp_amd/build.py.  The Python binding recomputes it from the shipped
// sources and refuses a library built from anything else (a stale .so pushed beside newer sources).
#include "gpudiff.h"
#include "gpudiff_synth.h"

#ifndef GPUDIFF_BUILD_ID
#error "build through kcp_amd/build.py: GPUDIFF_BUILD_ID is the sources' content hash"
#endif

extern "C" const char* gpudiff_build_id(void) { return GPUDIFF_BUILD_ID; }
extern "C" const char* gpudiff_synth_build_id(void) { return GPUDIFF_BUILD_ID; }
