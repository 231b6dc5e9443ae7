// bitop3_order.hip -- which operand of v_bitop3_b32 is the high bit of the truth-table index.
// With a = 0xF0.., b = 0xCC.., c = 0xAA.., the result equals the table iff index = 4a + 2b + c.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k(unsigned *o, unsigned a, unsigned b, unsigned c)
{
    o[0] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xEA);
    o[1] = __builtin_amdgcn_bitop3_b32(a, b, c, 0x6C);
}

int main()
{
    unsigned *o, h[2];
    if (hipMalloc(&o, 8) != hipSuccess)
        return 1;
    k<<<1, 1>>>(o, 0xF0F0F0F0u, 0xCCCCCCCCu, 0xAAAAAAAAu);
    if (hipMemcpy(h, o, 8, hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    printf("bitop3(F0,CC,AA,0xEA) = %08x  bitop3(...,0x6C) = %08x\n", h[0], h[1]);
    return 0;
}
