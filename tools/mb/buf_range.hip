// buf_range.hip -- how the buffer range check treats soffset and a dwordx4 that straddles
// num_records (raw buffer, stride 0), for global->VGPR loads and LDS-DMA loads.
// Build: hipcc -O3 --offload-arch=gfx950 buf_range.hip -o buf_range
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

// lane 0 loads 16 bytes at voffset vo + soffset so from a descriptor of nrec bytes
__global__ void probe(const unsigned *buf, unsigned nrec, unsigned vo, unsigned so, unsigned *out)
{
    __shared__ unsigned lds[64 * 4];
    const uint64_t b = reinterpret_cast<uint64_t>(buf);
    v4i rs;
    rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(b)));
    rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(b >> 32) & 0xFFFF));
    rs.z = __builtin_amdgcn_readfirstlane(int(nrec));
    rs.w = 0x00020000;
    const unsigned sso = __builtin_amdgcn_readfirstlane(so);
    v4i r;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(vo), "s"(rs), "s"(sso) : "memory");
    for (int i = threadIdx.x; i < 256; i += 64) lds[i] = 0xEEEEEEEE;
    __syncthreads();
    const unsigned m = __builtin_amdgcn_readfirstlane(unsigned(reinterpret_cast<uintptr_t>(lds)));
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_waitcnt vmcnt(0)\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(vo), "s"(rs), "s"(m), "s"(sso) : "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
        out[4] = lds[0]; out[5] = lds[1]; out[6] = lds[2]; out[7] = lds[3];
    }
}

int main()
{
    unsigned h[64];
    for (int i = 0; i < 64; i++) h[i] = 0x1000 + i;
    unsigned *d, *o;
    CK(hipMalloc(&d, sizeof h));
    CK(hipMalloc(&o, 64));
    CK(hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice));
    struct C { const char *what; unsigned nrec, vo, so; } cs[] = {
        {"in range            ", 256, 16, 0},
        {"straddle by 8 bytes ", 24, 16, 0},
        {"straddle by 4 bytes ", 28, 16, 0},
        {"past end            ", 16, 16, 0},
        {"soffset, v+s in     ", 256, 0, 16},
        {"soffset, v+s past   ", 16, 0, 16},
        {"soffset, v+s strad 8", 24, 0, 16},
    };
    for (auto &c : cs) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, c.nrec, c.vo, c.so, o);
        CK(hipDeviceSynchronize());
        unsigned r[8];
        CK(hipMemcpy(r, o, 32, hipMemcpyDeviceToHost));
        printf("%s nrec %3u vo %2u so %2u | vgpr %08x %08x %08x %08x | lds %08x %08x %08x %08x\n", c.what, c.nrec, c.vo, c.so,
               r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
    }
    return 0;
}
