// Diagnostic build of attention.hip with in-kernel cycle stamps (see stamp_gemm.hip).
#define MICLIP_STAMPS 1
#include "../../aihab-clip_amd/csrc/attention.hip"
#include "stamp_buf.h"
