// Diagnostic build of gemm.hip with in-kernel cycle stamps (MICLIP_STAMPS,
// common.h). Linked with the library's other objects into
// build/stamps/libstamp_gemm.so by `make stamps`; driven by scripts/stamps/run.py.
#define MICLIP_STAMPS 1
#include "../../aihab-clip_amd/csrc/gemm.hip"
#include "stamp_buf.h"
