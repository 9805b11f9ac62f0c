// Exhaustive check of the fast correctly-rounded reciprocal / square root used by the
// step kernel (pob_math.h) against IEEE 1/x and sqrt(x) on every float32 bit pattern in
// the fast-path range.  Prints mismatch counts; exit status 1 on any mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../po-brax_amd/csrc/pob_math.h"

__global__ void k_check(uint32_t hi_start, unsigned long long *bad, uint32_t *first) {
  const uint64_t idx = (uint64_t)hi_start * 65536u + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t bits = (uint32_t)idx;
  const float x = __uint_as_float(bits);
  if (pob_fast_range(x)) {
    const float r_ref = 1.0f / x, r = pob_rcp(x);
    if (__float_as_uint(r) != __float_as_uint(r_ref)) { atomicAdd(&bad[0], 1ull); atomicCAS(&first[0], 0u, bits); }
    if (x > 0.0f) {
      const float s_ref = sqrtf(x), s = pob_sqrt(x);
      if (__float_as_uint(s) != __float_as_uint(s_ref)) { atomicAdd(&bad[1], 1ull); atomicCAS(&first[1], 0u, bits); }
    }
  }
}

int main() {
  unsigned long long *bad; uint32_t *first;
  hipMalloc(&bad, 16); hipMalloc(&first, 8);
  hipMemset(bad, 0, 16); hipMemset(first, 0, 8);
  for (uint32_t hs = 0; hs < 65536u; hs += 1024u)
    for (uint32_t h = hs; h < hs + 1024u; ++h) hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, 0, h, bad, first);
  unsigned long long hb[2]; uint32_t hf[2];
  hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost); hipMemcpy(hf, first, 8, hipMemcpyDeviceToHost);
  printf("rcp mismatches %llu (first 0x%08x)  sqrt mismatches %llu (first 0x%08x)\n", hb[0], hf[0], hb[1], hf[1]);
  return (hb[0] || hb[1]) ? 1 : 0;
}
