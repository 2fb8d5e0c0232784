// probe_oob.hip -- how a raw buffer dwordx4 load that straddles the resource's end behaves on
// gfx950 (per dword, or the whole load zeroed).  Tooling, not product.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned* p, unsigned* o) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 100, 0x00020000);
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, 92u + 4u * threadIdx.x, 0, 0);  // lane 0: bytes 92..108
    o[4 * threadIdx.x + 0] = v.x; o[4 * threadIdx.x + 1] = v.y; o[4 * threadIdx.x + 2] = v.z; o[4 * threadIdx.x + 3] = v.w;
}
int main() {
    unsigned h[64], *d, *o, ho[16];
    for (int i = 0; i < 64; ++i) h[i] = 0x1000u + i;
    hipMalloc(&d, 256); hipMalloc(&o, 64);
    hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(4), 0, 0, d, o);
    hipMemcpy(ho, o, 64, hipMemcpyDeviceToHost);
    for (int l = 0; l < 4; ++l) printf("offset %d: %x %x %x %x\n", 92 + 4 * l, ho[4 * l], ho[4 * l + 1], ho[4 * l + 2], ho[4 * l + 3]);
    return 0;
}
