// The stamp buffer of one diagnostic library and its host accessors.
#pragma once
__device__ unsigned long long miclip_stamp_buf[1 << 17];

extern "C" int miclip_stamps_words() { return 1 << 17; }
extern "C" int miclip_stamps_clear(void* stream) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(miclip_stamp_buf)) != hipSuccess) return 1;
  return hipMemsetAsync(p, 0, sizeof(unsigned long long) << 17, (hipStream_t)stream) != hipSuccess;
}
extern "C" int miclip_stamps_read(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(miclip_stamp_buf), sizeof(unsigned long long) << 17) !=
         hipSuccess;
}
