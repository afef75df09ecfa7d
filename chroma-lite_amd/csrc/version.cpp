// version.cpp -- the library's identity: ABI version and the sha of the sources
// it was built from (tools/source_sha.py, written to _build/source_sha.h by the
// Makefile), so a prebuilt .so that travels with the tree can be checked against it.
#include "../../include/chroma_amd.h"
#include "source_sha.h"

extern "C" int chr_version(void) { return 1; }
extern "C" const char *chr_source_sha(void) { return CHR_SOURCE_SHA; }
