// Probe: do buffer_load_dword (VGPR and LDS-DMA) and global_load_lds_dword
// return the right bytes from byte-unaligned addresses on gfx950?
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/unaligned_lds.hip -o tools/ubench/unaligned_lds
#include <cstring>
#include <hip/hip_runtime.h>
__global__ void k(const unsigned char *g, unsigned *out, int o) {
    __shared__ unsigned lds[256];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, 0x7FFFFFF0, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, threadIdx.x * 4 + o, 0, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(g + threadIdx.x*4 + o), (__attribute__((address_space(3))) void*)(lds + 64), 4, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    out[threadIdx.x] = lds[threadIdx.x];
    out[64 + threadIdx.x] = lds[64 + threadIdx.x];
    out[128 + threadIdx.x] = __builtin_amdgcn_raw_buffer_load_b32(r, threadIdx.x * 4 + o, 0, 0);
}
#include <cstdio>
int main() {
    unsigned char h[1024]; for (int i = 0; i < 1024; ++i) h[i] = (unsigned char)(i * 7 + 3);
    unsigned char *g; unsigned *o; hipMalloc(&g, 1024); hipMalloc(&o, 192 * 4);
    hipMemcpy(g, h, 1024, hipMemcpyHostToDevice);
    for (int off = 0; off < 4; ++off) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, g, o, off);
        unsigned r[192]; hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
        int bad[3] = {0, 0, 0};
        for (int t = 0; t < 64; ++t) {
            unsigned e; memcpy(&e, h + 4 * t + off, 4);
            for (int k2 = 0; k2 < 3; ++k2) bad[k2] += r[64 * k2 + t] != e;
        }
        printf("offset %d: buffer_lds bad %d, global_lds bad %d, buffer_vgpr bad %d (lane1: %08x %08x %08x)\n", off, bad[0], bad[1], bad[2], r[1], r[65], r[129]);
    }
    return 0;
}
