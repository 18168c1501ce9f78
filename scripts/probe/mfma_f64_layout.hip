// Empirical lane layout of v_mfma_f64_16x16x4f64: D = A(16x4) * B(4x16).
// A[i][k] = 1 if (i,k) == (ia,ka) else 0, B[k][j] = 1 if (k,j) == (ka,jb): D has a single 1 at (ia,jb).
// Operands are fed assuming A lane l = A[l%16][l/16], B lane l = B[l/16][l%16]; the
// kernel reports which (lane, reg) receives the 1 for every (ia, jb).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));
__global__ void probe(int ia, int ka, int jb, int* out) {
  const int l = threadIdx.x;
  const double a = ((l % 16) == ia && (l / 16) == ka) ? 1.0 : 0.0;
  const double b = ((l / 16) == ka && (l % 16) == jb) ? 1.0 : 0.0;
  dbl4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int q = 0; q < 4; ++q)
    if (c[q] != 0.0) { out[0] = l; out[1] = q; out[2] = (int)c[q]; }
}
int main() {
  int* d; hipMalloc(&d, 16);
  int bad = 0;
  for (int ia = 0; ia < 16; ++ia)
    for (int jb = 0; jb < 16; ++jb) {
      int h[3] = {-1, -1, -1};
      hipMemcpy(d, h, 12, hipMemcpyHostToDevice);
      probe<<<1, 64>>>(ia, (ia + jb) % 4, jb, d);
      hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
      const int exp_l = jb + 16 * (ia / 4), exp_q = ia % 4;
      if (h[0] != exp_l || h[1] != exp_q) {
        if (bad < 20) printf("D[%d][%d]: lane %d reg %d (assumed lane %d reg %d)\n", ia, jb, h[0], h[1], exp_l, exp_q);
        ++bad;
      }
    }
  printf("mismatches: %d of 256\n", bad);
  return bad ? 1 : 0;
}
