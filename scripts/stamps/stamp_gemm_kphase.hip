// Diagnostic build of gemm.hip: the persistent kernel's main-loop phases split into
// stamp segments 1-7 (MICLIP_PSTAMP in gemm256s_kernel: 1 fragment reads incl. their
// latency -- the stamp's own s_memtime waits on the LDS counter --, 2 LDS-DMA issue,
// 3 lgkmcnt wait, 4 barrier before the MFMAs, 5 MFMA issue, 6 vmcnt wait, 7 the
// closing barrier); every other stamp of the kernel folds into segment 0.
// scripts/stamps/run.py gemm --phases prints them under these names.
#define MICLIP_STAMPS 1
#include "../../aihab-clip_amd/csrc/common.h"
#define MICLIP_STAMP_ACC(i)                                                            \
  do {                                                                                 \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();                        \
    st_.a##i += n_ - st_.t;                                                            \
    st_.t = n_;                                                                        \
  } while (0)
#undef MICLIP_STAMP
#define MICLIP_STAMP(i) MICLIP_STAMP_ACC(0)
#define MICLIP_PSTAMP(i) MICLIP_STAMP_ACC(i)
#include "../../aihab-clip_amd/csrc/gemm.hip"
#include "stamp_buf.h"
