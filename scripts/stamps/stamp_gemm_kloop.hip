// Diagnostic build of gemm.hip: stamps as stamp_gemm.hip, plus the persistent
// kernel's main-loop vmcnt waits as segment 6 (scripts/stamps/run.py prints it
// under "epi_barrier"; with this library read it as "K-loop vmcnt wait").
#define MICLIP_STAMPS 1
#define MICLIP_STAMPS_KLOOP 1
#include "../../aihab-clip_amd/csrc/gemm.hip"
#include "stamp_buf.h"
