"""MetaData packs on the GPU entry points: the format of MetaDataPack / MetaDataUnpack
(libbrb_core/data/utils/meta_data.c:104-328, libbrb_data.h:291-330, LP64), built and checked many at
a time.  The mmap'd file cache (ev_kq_file_mapped.c:2493, :2869) and the encrypted K/V files keep
their objects in this format, so a cache warm-up validates thousands of packs at once.

A pack is a 64-byte header {int version = 0; int item_count; unsigned long size; "BRB_META"; the MD5
of the items' data (MetaDataHeaderLoadData, :397-433); 24 zero bytes}, then per item
{unsigned long item_id, item_sub_id, sz; sz data bytes; 0x1F}; size = sum of (sz + 24 + 1).

pack_batch lays packs out back to back on the host and computes every header digest with one
BRB_MD5BatchSegments call whose segments are the item data inside the packed buffer itself;
unpack_batch is BRB_MetaDataUnpackBatch (one GPU lane per pack; reference return codes and
MetaDataUnpackerInfo fields, quirks included -- include/brb_crypto.h).  items() lists a pack's items
on the host, for packs unpack_batch accepted."""
import struct

import numpy as np

from . import crypto

HEADER = 64
ITEM_RAW = 24
MAGIC = b"BRB_META"
CANARY = 0x1F
UNPACK_SUCCESS = 7
UNPACK_CODES = {0: "FAILED_INVALID_HEADER_MAGIC", 1: "FAILED_UNINITIALIZED", 2: "FAILED_NO_RAWDATA",
                3: "FAILED_CORRUPTED_CANARY", 4: "FAILED_DIGEST_INVALID", 5: "FAILED_NEED_MORE_DATA_METAITEM",
                6: "FAILED_NEED_MORE_DATA_OBJECT", 7: "SUCCESS"}   # MetaDataUnpackReturnCode, libbrb_data.h:299-310


def pack_size(items) -> int:
    return HEADER + sum(ITEM_RAW + len(d) + 1 for _, _, d in items)


def pack_batch(packs):
    """MetaDataPack of every MetaData in `packs` (each a list of (item_id, item_sub_id, data bytes)).
    Returns (buf, offsets, lengths): pack i is buf[offsets[i] : offsets[i] + lengths[i]]."""
    sizes = np.array([pack_size(items) for items in packs], np.uint64)
    offsets = np.zeros(len(packs), np.uint64)
    if len(packs) > 1:
        offsets[1:] = np.cumsum(sizes)[:-1]
    buf = np.zeros(int(sizes.sum()) if len(packs) else 1, np.uint8)
    seg_off, seg_len, first = [], [], [0]
    for p, items in enumerate(packs):
        o = int(offsets[p])
        body = sum(ITEM_RAW + len(d) + 1 for _, _, d in items)
        buf[o:o + 24] = np.frombuffer(struct.pack("<iiQ8s", 0, len(items), body, MAGIC), np.uint8)
        o += HEADER
        for item_id, sub_id, data in items:
            buf[o:o + ITEM_RAW] = np.frombuffer(struct.pack("<QQQ", item_id, sub_id, len(data)), np.uint8)
            o += ITEM_RAW
            seg_off.append(o)
            seg_len.append(len(data))
            buf[o:o + len(data)] = np.frombuffer(data, np.uint8)
            o += len(data)
            buf[o] = CANARY
            o += 1
        first.append(len(seg_off))
    if len(packs):
        digests = crypto.md5_batch_segments(buf, np.array(seg_off, np.uint64), np.array(seg_len, np.uint32),
                                            np.array(first, np.uint64))
        for p in range(len(packs)):
            o = int(offsets[p]) + 24
            buf[o:o + 16] = digests[p]
    return buf, offsets, sizes.astype(np.uint32)


def unpack_batch(buf, offsets, lengths, stream=None, all_devices=False):
    """BRB_MetaDataUnpackBatch: one BRB_MetaDataUnpackInfo (error_code, item_count, cur_offset,
    cur_remaining, cur_needed) per pack, error_code a MetaDataUnpackReturnCode (7 = SUCCESS)."""
    return crypto.metadata_unpack_batch(buf, np.asarray(offsets, np.uint64), np.asarray(lengths, np.uint32),
                                        stream=stream, all_devices=all_devices)


def items(pack: bytes):
    """The (item_id, item_sub_id, data) items of a pack unpack_batch accepted (MetaDataItemAdd order)."""
    count = struct.unpack_from("<i", pack, 4)[0]
    out, o = [], HEADER
    for _ in range(max(count, 0)):
        if o == len(pack):
            break
        item_id, sub_id, sz = struct.unpack_from("<QQQ", pack, o)
        o += ITEM_RAW
        out.append((item_id, sub_id, bytes(pack[o:o + sz])))
        o += sz + 1
    return out
