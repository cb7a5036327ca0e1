// Diagnostic (GPU box only): what a multi-dword buffer access does when it
// straddles the descriptor's num_records, or starts below 0 (a wrapped
// offset).  Does the range check drop / zero the whole access, or each dword?
//   hipcc --offload-arch=gfx950 -O3 tools/buf_probe.hip -o tools/buf_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(uint32_t* buf, uint32_t* out) {
    if (threadIdx.x != 0) return;
    // descriptor over buf[4..9]: 24 bytes
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf + 4, (short)0, 24, 0x00020000);
    const u32x4 v = {0xA0u, 0xA1u, 0xA2u, 0xA3u};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, 16, 0, 0);           // dwords 4,5 in, 6,7 past the end
    const u32x4 w = {0xB0u, 0xB1u, 0xB2u, 0xB3u};
    __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)0xFFFFFFF8u, 0, 0);  // dwords -2,-1 below, 0,1 in
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, 16, 0, 0);
    const u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(r, (int)0xFFFFFFF8u, 0, 0);
    out[0] = x.x; out[1] = x.y; out[2] = x.z; out[3] = x.w;
    out[4] = y.x; out[5] = y.y; out[6] = y.z; out[7] = y.w;
    // a 64-bit access half past the end
    const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(buf + 16, (short)0, 4, 0x00020000);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 z = {0xC0u, 0xC1u};
    __builtin_amdgcn_raw_buffer_store_b64(z, r2, 0, 0, 0);
}

int main() {
    uint32_t *buf, *out;
    if (hipMalloc(&buf, 256) || hipMalloc(&out, 64)) return 1;
    (void)hipMemset(buf, 0x11, 256);
    (void)hipMemset(out, 0x22, 64);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, out);
    uint32_t hb[32], ho[16];
    if (hipMemcpy(hb, buf, 128, hipMemcpyDeviceToHost) || hipMemcpy(ho, out, 64, hipMemcpyDeviceToHost)) return 1;
    printf("buf[0..19] (descriptor over 4..9; store16 at 8..11 [4 in range 2 past]; store16 at 2..5 [2 below]; store8 at 16,17 with 4-byte range):\n");
    for (int i = 0; i < 20; ++i) printf(" %2d:%08x%s", i, hb[i], i % 5 == 4 ? "\n" : "");
    printf("load16 at 8..11: %08x %08x %08x %08x\n", ho[0], ho[1], ho[2], ho[3]);
    printf("load16 at 2..5 : %08x %08x %08x %08x\n", ho[4], ho[5], ho[6], ho[7]);
    return 0;
}
