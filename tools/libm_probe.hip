// libm_probe.hip — how often do gfx950 OCML double transcendentals differ
// from the host's glibc libm (which the reference's CPU build calls)?
// Measurement tool only (decides how the rare exact path evaluates them).
//   hipcc -O2 --offload-arch=gfx950 tools/libm_probe.hip -o /tmp/libm_probe && /tmp/libm_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#pragma clang fp contract(off)

__global__ void probe(const double* x, double* out, int n, int fn) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = x[i];
  double r;
  switch (fn) {
    case 0: r = exp(v); break;
    case 1: r = log(v); break;
    case 2: r = sin(v); break;
    case 3: r = pow(v, 3.0); break;
    case 4: r = sqrt(v); break;
    default: r = 1.0 / v; break;
  }
  out[i] = r;
}

static double host_fn(int fn, double v) {
  switch (fn) {
    case 0: return exp(v);
    case 1: return log(v);
    case 2: return sin(v);
    case 3: return pow(v, 3.0);
    case 4: return sqrt(v);
    default: return 1.0 / v;
  }
}

int main() {
  const int n = 1 << 22;
  const char* names[] = {"exp[-745,5]", "log(0,10]", "sin[0,60]", "pow(x,3)", "sqrt", "1/x"};
  double* hx = (double*)malloc(n * sizeof(double));
  double* hy = (double*)malloc(n * sizeof(double));
  double *dx, *dy;
  hipMalloc(&dx, n * sizeof(double));
  hipMalloc(&dy, n * sizeof(double));
  srand48(12345);
  for (int fn = 0; fn < 6; ++fn) {
    for (int i = 0; i < n; ++i) {
      double u = drand48();
      hx[i] = fn == 0 ? -745.0 + 750.0 * u : fn == 1 ? 1e-300 + 10.0 * u
            : fn == 2 ? 60.0 * u : fn == 3 ? 1e-3 + 3.0 * u : 1e-3 + 10.0 * u;
    }
    hipMemcpy(dx, hx, n * sizeof(double), hipMemcpyHostToDevice);
    probe<<<n / 256, 256>>>(dx, dy, n, fn);
    hipMemcpy(hy, dy, n * sizeof(double), hipMemcpyDeviceToHost);
    long diff = 0, diff2 = 0;
    for (int i = 0; i < n; ++i) {
      double h = host_fn(fn, hx[i]);
      long long a, b;
      memcpy(&a, &h, 8);
      memcpy(&b, &hy[i], 8);
      long long d = a > b ? a - b : b - a;
      if (d) ++diff;
      if (d > 1) ++diff2;
    }
    printf("{\"fn\": \"%s\", \"n\": %d, \"differ\": %.6e, \"differ_gt_1ulp\": %.6e}\n", names[fn], n,
           (double)diff / n, (double)diff2 / n);
  }
  return 0;
}
