// Diagnostic: device libm (ocml) vs host glibc, max |ulp| difference per function.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../flow-state_amd/csrc/physics_device.h"

__global__ void k(const double *x, int n, double *o) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = x[i];
    o[6 * i + 0] = tanh(v);
    o[6 * i + 1] = exp(v);
    o[6 * i + 2] = fs::pow6(1.0 / (fabs(v) + 0.5));
    o[6 * i + 3] = sqrt(fabs(v) * 3.0);
    o[6 * i + 4] = fmod(v * 13.0, 46.188);
    o[6 * i + 5] = fs::np_remainder(v * 17.0, 46.188);
}

static int64_t ulpd(double a, double b) {
    if (a == b) return 0;
    int64_t ia, ib;
    memcpy(&ia, &a, 8); memcpy(&ib, &b, 8);
    if (ia < 0) ia = INT64_MIN - ia;
    if (ib < 0) ib = INT64_MIN - ib;
    return llabs(ia - ib);
}

int main() {
    const int n = 1 << 20;
    std::vector<double> x(n), o(6 * n);
    srand(1);
    for (int i = 0; i < n; ++i) x[i] = ((double)rand() / RAND_MAX - 0.5) * 10.0;
    double *dx, *dout;
    hipMalloc(&dx, n * 8); hipMalloc(&dout, 6 * n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dx, n, dout);
    hipMemcpy(o.data(), dout, 6 * n * 8, hipMemcpyDeviceToHost);
    const char *names[6] = {"tanh", "exp", "pow6(1/r) vs pow", "sqrt", "fmod", "np_remainder"};
    for (int f = 0; f < 6; ++f) {
        int64_t mx = 0; long cnt = 0; double worst = 0;
        for (int i = 0; i < n; ++i) {
            double v = x[i], h;
            switch (f) {
            case 0: h = tanh(v); break;
            case 1: h = exp(v); break;
            case 2: h = pow(1.0 / (fabs(v) + 0.5), 6.0); break;
            case 3: h = sqrt(fabs(v) * 3.0); break;
            case 4: h = fmod(v * 13.0, 46.188); break;
            default: { double a = v * 17.0, b = 46.188, m = fmod(a, b); if (m != 0.0) { if ((b < 0) != (m < 0)) m += b; } else m = copysign(0.0, b); h = m; }
            }
            int64_t u = ulpd(h, o[6 * i + f]);
            if (u) cnt++;
            if (u > mx) { mx = u; worst = v; }
        }
        printf("%-18s max_ulp=%lld  n_diff=%ld/%d  worst_x=%.17g\n", names[f], (long long)mx, cnt, n, worst);
    }
    return 0;
}
