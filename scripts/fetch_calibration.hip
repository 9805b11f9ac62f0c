// fetch_calibration.hip -- calibrate rocprofv3's FETCH_SIZE on the step kernel's own load
// pattern (MI355X_MICROARCH.md §HBM: the counter reads exactly 1/2 of the bytes of a 16-B/lane
// streaming read; other access widths are uncalibrated).
//
// Three kernels read qp-shaped arrays of B envs (AntHeavenHell: N = 14 bodies, pos / vel / ang
// (B, N, 3), rot (B, N, 4), float32) whose byte counts are known:
//   k_rows    the step kernel's pattern (pob_quad.h / pob_kernels.hip per-lane loads): four lanes
//             per env, lane k reads the rows of bodies 0, 2k + 1, 2k + 2 (12-B / 16-B row loads);
//             the 9 dynamic bodies' rows cover 108 of every 168-B pos row, so EVERY 64-B / 128-B
//             line of the arrays is touched: the lines' bytes = the arrays' bytes
//   k_stream  the guide's calibrated case over the same arrays: 16 B per lane, fully coalesced
//   k_dense   the same 12-B / 16-B per-lane row loads over arrays holding ONLY the 9 dynamic
//             rows (B, 9, c): what a body-major / dense layout would read
// Each writes one float per env (a checksum, 262 KB at B = 65 536).  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calibration
// and compare FETCH_SIZE (KiB) per dispatch with the printed byte counts.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                                   \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); }     \
  } while (0)

struct f3 { float x, y, z; };

__device__ __forceinline__ float ld3(const float *p) {
  const f3 v = *reinterpret_cast<const f3 *>(p);
  return v.x + v.y + v.z;
}
__device__ __forceinline__ float ld4(const float *p) {
  const float4 v = *reinterpret_cast<const float4 *>(p);
  return v.x + v.y + v.z + v.w;
}

// NB: bodies per env row (the arrays' N); the lane reads bodies 0, 2k+1, 2k+2 (< 9)
template <int NB>
__global__ __launch_bounds__(256) void k_rows(const float *pos, const float *rot, const float *vel, const float *ang,
                                             int B, float *out) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = gid >> 2, k = gid & 3;
  if (b >= B) return;
  float s = 0.0f;
  const int g[3] = {0, 2 * k + 1, 2 * k + 2};
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const size_t r3 = ((size_t)b * NB + g[l]) * 3, r4 = ((size_t)b * NB + g[l]) * 4;
    s += ld3(pos + r3) + ld4(rot + r4) + ld3(vel + r3) + ld3(ang + r3);
  }
  out[gid] = s;
}

__global__ __launch_bounds__(256) void k_stream(const float4 *p, size_t n4, float *out) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float s = 0.0f;
  for (size_t i = gid; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = p[i];
    s += v.x + v.y + v.z + v.w;
  }
  out[gid] = s;
}

int main(int argc, char **argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 65536;
  const int N = 14, ND = 9;
  const size_t n3 = (size_t)B * N * 3, n4 = (size_t)B * N * 4;
  const size_t d3 = (size_t)B * ND * 3, d4 = (size_t)B * ND * 4;
  const size_t full = (3 * n3 + n4) * sizeof(float), dense = (3 * d3 + d4) * sizeof(float);
  float *buf, *dbuf, *out;
  CHECK(hipMalloc(&buf, full));
  CHECK(hipMalloc(&dbuf, dense));
  CHECK(hipMalloc(&out, sizeof(float) * (size_t)B * 4 + sizeof(float) * 1024 * 256));
  CHECK(hipMemset(buf, 0, full));
  CHECK(hipMemset(dbuf, 0, dense));
  // a 512 MiB scrub buffer: each timed kernel starts with the arrays out of L2 and the 256 MiB
  // Infinity Cache
  const size_t scrub_n = (size_t)512 << 20;
  char *scrub;
  CHECK(hipMalloc(&scrub, scrub_n));
  float *pos = buf, *vel = buf + n3, *ang = buf + 2 * n3, *rot = buf + 3 * n3;
  float *dpos = dbuf, *dvel = dbuf + d3, *dang = dbuf + 2 * d3, *drot = dbuf + 3 * d3;
  const int blocks = (4 * B + 255) / 256;
  printf("{\"B\": %d, \"bytes_full_arrays\": %zu, \"bytes_dense_dynamic_rows\": %zu, "
         "\"bytes_algorithmic_dynamic_rows\": %zu}\n", B, full, dense, (size_t)B * ND * 13 * sizeof(float));
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipMemset(scrub, rep, scrub_n));
    hipLaunchKernelGGL(k_rows<14>, dim3(blocks), dim3(256), 0, 0, pos, rot, vel, ang, B, out);
    CHECK(hipMemset(scrub, rep + 1, scrub_n));
    hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, (const float4 *)buf, full / 16, out);
    CHECK(hipMemset(scrub, rep + 2, scrub_n));
    hipLaunchKernelGGL(k_rows<9>, dim3(blocks), dim3(256), 0, 0, dpos, drot, dvel, dang, B, out);
  }
  CHECK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
