// Probe of fx_scan_common.h's cross-lane helpers (tests/test_lane_swap.py).
#include "fx_scan_common.h"

__global__ void k_lane_probe(int* out) {
    const int lane = threadIdx.x & 63;
    const int x = (lane * 7 + 3) % 11;
    int ex, tot;
    fx::quad_prefix(x, lane, ex, tot);
    out[lane] = fx::lane_xor16(x, lane);
    out[64 + lane] = fx::lane_xor32(x, lane);
    out[128 + lane] = ex;
    out[192 + lane] = tot;
}

extern "C" int lane_probe(int* host_out) {
    int* d = nullptr;
    if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_lane_probe, dim3(1), dim3(64), 0, 0, d);
    int rc = hipMemcpy(host_out, d, 256 * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
    (void)hipFree(d);
    return rc;
}
