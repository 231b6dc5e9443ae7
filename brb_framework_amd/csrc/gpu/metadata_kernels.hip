// metadata_kernels.hip -- batched MetaDataUnpack (libbrb_core/data/utils/meta_data.c:145-328) over
// many MetaData packs (the mmap'd file cache and encrypted K/V files keep their
// objects as packs whose MD5 covers the items' data).
//
// One lane per pack.  A pack is one sequential byte stream -- header, then per item three 8-byte
// fields, the data, the 0x1F canary -- whose every position depends on the sizes before it, so the
// lane's loads form a chain.  The chain is kept off the critical path: the header comes with the
// first item's fields in one read, an item's data streams in 64-byte blocks with the next block in
// flight (brb_io::BlockSrc), and the 25 bytes after the data (the canary and the next item's
// fields) are loaded before the data is hashed (Ahead).  The data feeds the lane's MD5
// (md5_funnel.h).  The control flow and the
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

// N little-endian dwords of the pack from byte q (any alignment): the N + 1 aligned dwords that
// hold pack bytes are loaded together (the others read as 0), funnel-shifted, and bytes at or past
// `size` are zeroed.  Issued early, they land while the lane hashes the item before them.
template <int N>
struct Ahead {
    uint32_t d[N + 1];
    uint32_t sh;
    uint64_t q, size;

    BRB_DEV void issue(const uint8_t *base, uint64_t size_, uint64_t q_)
    {
        q = q_;
        size = size_;
        const uintptr_t a = reinterpret_cast<uintptr_t>(base) + q;
        const uint32_t *p = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
        sh = uint32_t(a & 3) * 8;
        const uint64_t first = q - (a & 3);                   // pack byte of dword 0 (may be q - 3 .. q)
#pragma unroll
        for (int i = 0; i < N + 1; i++) {
            // dword i starts at pack byte b (b in -3 .. -1, wrapped, for a dword that starts before
            // the pack): it is loaded iff it holds a pack byte
            const uint64_t b = first + 4 * uint64_t(i);
            d[i] = size && (b < size || b > ~uint64_t(0) - 3) ? ldg(p + i) : 0u;
        }
    }
    BRB_DEV uint32_t dw(int i) const                          // pack bytes q + 4i .. q + 4i + 3
    {
        const uint32_t v = __builtin_amdgcn_alignbit(d[i + 1], d[i], sh);
        const uint64_t at = q + 4 * uint64_t(i);
        if (at >= size)
            return 0u;
        const uint64_t left = size - at;
        return left >= 4 ? v : v & ((1u << (8 * uint32_t(left))) - 1u);
    }
    BRB_DEV uint64_t qw(int i) const { return uint64_t(dw(i)) | (uint64_t(dw(i + 1)) << 32); }
};

__global__ __launch_bounds__(kBlock) void metadata_unpack_kernel(const uint8_t *__restrict__ data,
                                                                 const uint64_t *__restrict__ offs,
                                                                 const uint32_t *__restrict__ lens, uint64_t n,
                                                                 BRB_MetaDataUnpackInfo *__restrict__ info)
{
    __shared__ __attribute__((aligned(8192))) uint32_t blk[kBlock / 64][brb_md5::kRingWords][64];   // 8 KiB per wave
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n)
        return;
    const uint8_t *base = data + offs[r];
    const uint64_t size = lens[r];
    int32_t code;
    uint32_t items = 0;
    uint64_t offset = 0, remaining = 0, needed = 0;   // cur_offset starts at the MemBuffer offset, 0

    // MetaDataHeader (libbrb_data.h:322-330) and the first item's three fields: bytes 0 .. 87
    Ahead<22> hd;
    hd.issue(base, size, 0);
    const int32_t item_count = int32_t(hd.dw(1));
    const uint64_t magic = hd.qw(4);
    const uint32_t dig[4] = {hd.dw(6), hd.dw(7), hd.dw(8), hd.dw(9)};
    if (magic != kMagic) {                                  // meta_data.c:183-195
        code = BRB_METADATA_UNPACK_FAILED_INVALID_HEADER_MAGIC;
    } else {
        offset = BRB_METADATA_HEADER_SIZE;                  // :198-199
        brb_md5::Funnel f;
        f.init(&blk[wave][0][lane]);
        code = BRB_METADATA_UNPACK_SUCCESS;
        uint64_t sz = hd.qw(20);                            // item 0's sz (bytes 80..87)
        for (int32_t i = 0; i < item_count; i++) {          // :202
            remaining = size - offset;                      // :213 (unsigned long)
            if (remaining < kItemStruct) {                  // :216-224
                needed = kItemStruct - remaining;
                code = BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_METAITEM;
                break;
            }
            offset += kItemRaw;                             // :227-232 (item_id, item_sub_id skipped)
            remaining -= kItemRaw;
            if (remaining < sz + 1 || sz > size) {          // :237-246 (sz > size: never read, see header)
                needed = sz + 1 - remaining;
                code = BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_OBJECT;
                break;
            }
            // the canary and the next item's fields (bytes offset + sz .. + 24) load while the data
            // is hashed; the data comes in 64-byte blocks with the next one in flight
            Ahead<7> nx;
            nx.issue(base, size, offset + sz);
            // The data is read from e = (bytes digested so far) mod 4 bytes before it (the item's
            // own fields, offset >= 88 > e), so its words fall on the digest's word boundaries: one
            // funnel shift per word (in BlockSrc) and no carry shifting (md5_funnel.h put16w); the
            // first word's e low bytes are the carried ones.  Here sz + 1 <= size - offset.
            const uint32_t e = f.nacc;
            const uint64_t n = sz + e;
            brb_io::BlockSrc bs;   // two blocks in flight (registers copied per block): 75.7 -> 81.4 us
            bs.init(base + offset - e, n);
            for (uint64_t c = 0; c < n; c += 64) {          // :249-254 BRB_MD5UpdateBig of the data
                uint32_t w[16];
                bs.fetch(w);
                if (c == 0)
                    w[0] = f.head(w[0]);
                const uint64_t left = n - c;
                if (left >= 64)
                    f.put16w(w);
                else
                    f.put_tail(w, uint32_t(left));
                f.pump();
            }
            if ((n & 63) == 0) {                            // ended on a whole block: nothing carried
                f.acc = 0;
                f.nacc = 0;
            }
            f.total += sz;
            offset += sz;
            remaining -= sz;
            if ((nx.dw(0) & 0xFFu) != 0x1Fu) {              // :258-268
                code = BRB_METADATA_UNPACK_FAILED_CORRUPTED_CANARY;
                break;
            }
            offset += 1;                                    // :271-277
            remaining -= 1;
            items++;
            if (offset == size)                             // :280-281
                break;
            // next item's sz: pack bytes offset + 16 .. + 23 = bytes 17 .. 24 of nx
            sz = uint64_t(__builtin_amdgcn_alignbit(nx.dw(5), nx.dw(4), 8)) |
                 (uint64_t(__builtin_amdgcn_alignbit(nx.dw(6), nx.dw(5), 8)) << 32);
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
