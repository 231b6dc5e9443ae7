// metadata_kernels.hip -- batched MetaDataUnpack (libbrb_core/data/utils/meta_data.c:145-328) over
// many MetaData packs (the mmap'd file cache and encrypted K/V files keep their
// objects as packs whose MD5 covers the items' data).
//
// One lane per pack.  A pack is one sequential byte stream -- header, then per item three 8-byte
// fields, the data, the 0x1F canary -- so the lane reads it front to back through brb_io::Src
// (aligned dword loads, a funnel shift, zeros past the pack) with a 0..7-byte carry for pieces that
// are not whole dwords, and feeds the item data to its MD5 (md5_funnel.h).  The control flow and the
// unsigned-long arithmetic of cur_offset / cur_remaining / cur_needed are the reference's; see
// include/brb_crypto.h for the two rules where the reference reads past its buffer.
#include "brb_kernels.h"
#include "byte_stream.h"
#include "md5_funnel.h"

namespace {

constexpr int kBlock = 256;
constexpr uint64_t kMagic = 0x4154454D5F425242ull;   // "BRB_META" as a little-endian unsigned long
constexpr uint64_t kItemStruct = 32;                  // sizeof(MetaDataItem): 3 unsigned longs + a pointer
constexpr uint64_t kItemRaw = 24;                     // METADATA_ITEM_RAW_SZ (libbrb_data.h:297)

// Sequential little-endian reads of 1..4 bytes (take) or 8 bytes (take64) from a byte range.
struct Reader {
    brb_io::Src src;
    uint64_t buf;       // bytes read from src and not yet taken, lowest first
    uint32_t nbuf;

    BRB_DEV void init(const uint8_t *a, uint64_t n)
    {
        src.init(a, n);
        buf = 0;
        nbuf = 0;
    }
    BRB_DEV uint32_t take(uint32_t k)
    {
        if (nbuf < k) {
            buf |= uint64_t(src.next()) << (8 * nbuf);
            nbuf += 4;
        }
        const uint32_t v = k == 4 ? uint32_t(buf) : uint32_t(buf) & ((1u << (8 * k)) - 1u);
        buf = k == 4 ? buf >> 32 : buf >> (8 * k);
        nbuf -= k;
        return v;
    }
    BRB_DEV uint64_t take64()
    {
        const uint64_t lo = take(4);
        return lo | (uint64_t(take(4)) << 32);
    }
};

__global__ __launch_bounds__(kBlock) void metadata_unpack_kernel(const uint8_t *__restrict__ data,
                                                                 const uint64_t *__restrict__ offs,
                                                                 const uint32_t *__restrict__ lens, uint64_t n,
                                                                 BRB_MetaDataUnpackInfo *__restrict__ info)
{
    __shared__ uint32_t blk[kBlock / 64][16][64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n)
        return;
    const uint64_t size = lens[r];
    Reader rd;
    rd.init(data + offs[r], size);
    int32_t code;
    uint32_t items = 0;
    uint64_t offset = 0, remaining = 0, needed = 0;   // cur_offset starts at the MemBuffer offset, 0

    // MetaDataHeader (libbrb_data.h:322-330): version, item_count, size, str, digest, reserved
    (void)rd.take(4);
    const int32_t item_count = int32_t(rd.take(4));
    (void)rd.take64();
    const uint64_t magic = rd.take64();
    uint32_t dig[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
        dig[i] = rd.take(4);
#pragma unroll
    for (int i = 0; i < 6; i++)
        (void)rd.take(4);
    if (magic != kMagic) {                                  // meta_data.c:183-195
        code = BRB_METADATA_UNPACK_FAILED_INVALID_HEADER_MAGIC;
    } else {
        offset = BRB_METADATA_HEADER_SIZE;                  // :198-199
        brb_md5::Funnel f;
        f.init(&blk[wave][0][lane]);
        code = BRB_METADATA_UNPACK_SUCCESS;
        for (int32_t i = 0; i < item_count; i++) {          // :202
            remaining = size - offset;                      // :213 (unsigned long)
            if (remaining < kItemStruct) {                  // :216-224
                needed = kItemStruct - remaining;
                code = BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_METAITEM;
                break;
            }
            (void)rd.take64();                              // item_id
            (void)rd.take64();                              // item_sub_id
            const uint64_t sz = rd.take64();
            offset += kItemRaw;                             // :227-232
            remaining -= kItemRaw;
            if (remaining < sz + 1 || sz > size) {          // :237-246 (sz > size: never read, see header)
                needed = sz + 1 - remaining;
                code = BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_OBJECT;
                break;
            }
            for (uint64_t c = 0; c < sz; c += 4) {          // :249-254 BRB_MD5UpdateBig of the data
                const uint32_t k = sz - c >= 4 ? 4u : uint32_t(sz - c);
                f.put(rd.take(k), k);
            }
            offset += sz;
            remaining -= sz;
            if (rd.take(1) != 0x1Fu) {                      // :258-268
                code = BRB_METADATA_UNPACK_FAILED_CORRUPTED_CANARY;
                break;
            }
            offset += 1;                                    // :271-277
            remaining -= 1;
            items++;
            if (offset == size)                             // :280-281
                break;
        }
        if (code == BRB_METADATA_UNPACK_SUCCESS) {          // :287-298
            const Md5State st = f.finish();
            if (st.a != dig[0] || st.b != dig[1] || st.c != dig[2] || st.d != dig[3])
                code = BRB_METADATA_UNPACK_FAILED_DIGEST_INVALID;
        }
    }
    BRB_MetaDataUnpackInfo o;
    o.error_code = code;
    o.item_count = items;
    o.cur_offset = offset;
    o.cur_remaining = remaining;
    o.cur_needed = needed;
    info[r] = o;
}

}  // namespace

namespace brb {

hipError_t launch_metadata_unpack(const uint8_t *data, const uint64_t *offs, const uint32_t *lens, uint64_t n,
                                  BRB_MetaDataUnpackInfo *info, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    metadata_unpack_kernel<<<unsigned((n + kBlock - 1) / kBlock), kBlock, 0, s>>>(data, offs, lens, n, info);
    return hipGetLastError();
}

}  // namespace brb
