// Probe: pob_mesh.h mesh_face on non-finite segments (NaN / inf end points) under both guard
// policies; prints every emitted contact (none expected: the oracle emits none).
#include "../po-brax_amd/csrc/pob_mesh.h"
#include <cstdio>

struct Out { int n; float tau[12], pen[12], d2[12]; };

template <class G>
__global__ void probe(const float *ab, Out *out, int ncase) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ncase) return;
  G g;
  const v3 A = V(ab[6 * i], ab[6 * i + 1], ab[6 * i + 2]), B = V(ab[6 * i + 3], ab[6 * i + 4], ab[6 * i + 5]);
  const float r = 0.08f, T = (r * r) * 1.00000095367431640625f;
  int n = 0;
  for (int f = 0; f < 6; ++f)
    mesh_face(g, f, A, B, true, 6.75f, 0.5f, 0.5f, r, T, [&](float tau, v3 nl, float pen) {
      if (n < 12) { out[i].tau[n] = tau; out[i].pen[n] = pen; out[i].d2[n] = nl.x; }
      ++n;
    });
  out[i].n = n;
}

int main() {
  const float nan = __builtin_nanf(""), inf = __builtin_inff();
  float h[6 * 8] = {nan, nan, nan, nan, nan, nan,   0.1f, 0.2f, 0.3f, nan, nan, nan,
                    nan, nan, nan, 0.1f, 0.2f, 0.3f, inf, inf, inf, inf, inf, inf,
                    nan, 0.2f, 0.3f, nan, 0.2f, 0.1f, 0.1f, 0.4f, 0.3f, 0.2f, 0.6f, 0.3f,
                    -inf, 0.f, 0.f, inf, 0.f, 0.f, 1e30f, 1e30f, 1e30f, -1e30f, -1e30f, -1e30f};
  const int nc = 8;
  float *dab; Out *dout; Out hout[nc];
  hipMalloc(&dab, sizeof(h)); hipMalloc(&dout, sizeof(hout));
  hipMemcpy(dab, h, sizeof(h), hipMemcpyHostToDevice);
  for (int pol = 0; pol < 2; ++pol) {
    hipMemset(dout, 0, sizeof(hout));
    if (pol == 0) probe<GuardBranch><<<1, 64>>>(dab, dout, nc);
    else probe<GuardAcc><<<1, 64>>>(dab, dout, nc);
    hipMemcpy(hout, dout, sizeof(hout), hipMemcpyDeviceToHost);
    for (int i = 0; i < nc; ++i) {
      printf("%s case %d: %d contacts", pol ? "GuardAcc" : "GuardBranch", i, hout[i].n);
      for (int k = 0; k < hout[i].n && k < 3; ++k) printf(" (tau %g pen %g)", hout[i].tau[k], hout[i].pen[k]);
      printf("\n");
    }
  }
  return 0;
}
