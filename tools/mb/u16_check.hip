// u16_check.hip -- which gfx950 16-bit integer ops leave a clean 16-bit value in a 32-bit VGPR?
// The RC4 generator (rc4_device.h) keeps its LDS byte addresses as 16-bit values (index << 8 |
// column) and advances them mod 2^16.  v_add_u16 / v_mad_u16 write the low half only (DESIGN §4.3:
// round 2's parity tests failed with them); the packed v_pk_add_u16 / v_pk_mad_u16 write both halves,
// the high half being the sum of the (zero) high halves.  Each op runs with a destination that holds
// garbage in its high half beforehand.
// Build: hipcc -O3 --offload-arch=gfx950 u16_check.hip -o u16_check
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(uint32_t *o, const uint32_t *a, const uint32_t *b)
{
    const uint32_t x = a[threadIdx.x], y = b[threadIdx.x];
    uint32_t r0 = 0xDEAD0000u | threadIdx.x, r1 = 0xBEEF0000u | threadIdx.x;
    uint32_t r2 = 0xDEAD0000u | threadIdx.x, r3 = 0xBEEF0000u | threadIdx.x;
    asm volatile("v_mad_u16 %0, %1, %2, %3" : "+v"(r0) : "v"(y), "s"(256u), "v"(x));
    asm volatile("v_add_u16_e32 %0, 0x100, %1" : "+v"(r1) : "v"(x));
    asm volatile("v_pk_mad_u16 %0, %1, %2, %3" : "+v"(r2) : "v"(y), "s"(256u), "v"(x));
    asm volatile("v_pk_add_u16 %0, %1, %2" : "+v"(r3) : "v"(x), "s"(256u));
    o[threadIdx.x] = r0;
    o[threadIdx.x + 64] = r1;
    o[threadIdx.x + 128] = r2;
    o[threadIdx.x + 192] = r3;
}

int main()
{
    uint32_t ha[64], hb[64], ho[256];
    for (int i = 0; i < 64; i++) { ha[i] = 0xFF00u + i; hb[i] = 3u * i + 1; }
    uint32_t *da, *db, *dout;
    if (hipMalloc(&da, 256) != hipSuccess || hipMalloc(&db, 256) != hipSuccess || hipMalloc(&dout, 1024) != hipSuccess ||
        hipMemcpy(da, ha, 256, hipMemcpyHostToDevice) != hipSuccess || hipMemcpy(db, hb, 256, hipMemcpyHostToDevice) != hipSuccess)
        return 1;
    k<<<1, 64>>>(dout, da, db);
    if (hipMemcpy(ho, dout, 1024, hipMemcpyDeviceToHost) != hipSuccess) { printf("HIP error\n"); return 1; }
    const char *name[4] = {"v_mad_u16", "v_add_u16", "v_pk_mad_u16", "v_pk_add_u16"};
    int bad_pk = 0;
    for (int op = 0; op < 4; op++) {
        int bad = 0;
        for (int i = 0; i < 64; i++) {
            const uint32_t want = (op & 1) ? (ha[i] + 256u) & 0xFFFFu : (ha[i] + (hb[i] << 8)) & 0xFFFFu;
            if (ho[64 * op + i] != want) {
                if (!bad)
                    printf("  %s lane %d: %08x (want %08x)\n", name[op], i, ho[64 * op + i], want);
                bad++;
            }
        }
        printf("%-13s %s\n", name[op], bad ? "leaves the high half (not a clean 16-bit result)" : "clean 16-bit result");
        if (op >= 2)
            bad_pk += bad;
    }
    return bad_pk ? 2 : 0;      // the generator uses the packed forms
}
