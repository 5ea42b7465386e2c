// Probe of the VALU cross-lane helpers of the scan and the refine
// (fx_device.h lane_xor<S>, sort64), checked
// against their definitions by tests/test_lane_swap.py.
#include "fx_scan_common.h"

// out[0 .. 6*64): lane_xor<1..32>(x); then lane ^ 48, lane ^ 7; then a
// sort64 of (key, id) with duplicate keys: keys and ids
__global__ void k_lane_probe(const float* keys_in, int* out, float* keys_out) {
    const int lane = threadIdx.x & 63;
    const int x = (lane * 7 + 3) % 11;
    out[0 * 64 + lane] = fx::lane_xor<1>(x, lane);
    out[1 * 64 + lane] = fx::lane_xor<2>(x, lane);
    out[2 * 64 + lane] = fx::lane_xor<4>(x, lane);
    out[3 * 64 + lane] = fx::lane_xor<8>(x, lane);
    out[4 * 64 + lane] = fx::lane_xor<16>(x, lane);
    out[5 * 64 + lane] = fx::lane_xor<32>(x, lane);
    // lane ^ 48 and lane ^ 7 as compositions
    out[6 * 64 + lane] = fx::lane_xor<16>(fx::lane_xor<32>(x, lane), lane);
    out[7 * 64 + lane] = fx::lane_xor<1>(fx::lane_xor<2>(fx::lane_xor<4>(x, lane), lane), lane);
    float d = keys_in[lane];
    int i = (lane * 37) % 64;
    fx::sort64(d, i, lane);
    keys_out[lane] = d;
    out[8 * 64 + lane] = i;
}

extern "C" int lane_probe(const float* host_keys, int* host_out, float* host_keys_out) {
    int* d = nullptr;
    float *kin = nullptr, *kout = nullptr;
    if (hipMalloc(&d, 9 * 64 * sizeof(int)) != hipSuccess) return 1;
    if (hipMalloc(&kin, 64 * 4) != hipSuccess || hipMalloc(&kout, 64 * 4) != hipSuccess) return 1;
    if (hipMemcpy(kin, host_keys, 64 * 4, hipMemcpyHostToDevice) != hipSuccess) return 2;
    hipLaunchKernelGGL(k_lane_probe, dim3(1), dim3(64), 0, 0, kin, d, kout);
    int rc = hipMemcpy(host_out, d, 9 * 64 * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess ? 0 : 3;
    if (rc == 0 && hipMemcpy(host_keys_out, kout, 64 * 4, hipMemcpyDeviceToHost) != hipSuccess) rc = 4;
    (void)hipFree(d);
    (void)hipFree(kin);
    (void)hipFree(kout);
    return rc;
}
