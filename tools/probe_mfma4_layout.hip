// tools/probe_mfma4_layout.hip -- the operand / result lane layout of
// v_mfma_f64_4x4x4_4b_f64 on gfx950: for every A lane (B = ones) and every B
// lane (A = ones), which D lanes receive it.
//   hipcc --offload-arch=gfx950 -O3 tools/probe_mfma4_layout.hip -o /tmp/probe4 && /tmp/probe4
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void kprobe(int which, int t, double *out) {
    const int lane = threadIdx.x;
    const double hot = lane == t ? 1.0 : 0.0;
    const double a = which == 0 ? hot : 1.0, b = which == 0 ? 1.0 : hot;
    out[lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}

int main() {
    double *d, h[64];
    if (hipMalloc(&d, 64 * sizeof(double)) != hipSuccess) return 1;
    for (int which = 0; which < 2; ++which)
        for (int t = 0; t < 64; ++t) {
            hipLaunchKernelGGL(kprobe, dim3(1), dim3(64), 0, 0, which, t, d);
            if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
            printf("%s lane %2d ->", which == 0 ? "A" : "B", t);
            for (int l = 0; l < 64; ++l)
                if (h[l] != 0.0) printf(" %d", l);
            printf("\n");
        }
    hipFree(d);
    return 0;
}
