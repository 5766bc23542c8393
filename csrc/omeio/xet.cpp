// Xet CAS chunk decoding for the model agent's Hugging Face downloads (reference pkg/xet: the
// Rust crate drives xet-core's FileDownloader; here the protocol lives in
// ome_amd/storage/xet.py and only the byte-level work is native).
//
// A file is reconstructed from "terms" = chunk ranges of content-addressed xorbs.  Each fetched
// xorb byte range is a run of chunks:
//   header (8 B): version u8 | compressed length u24 LE | scheme u8 | uncompressed length u24 LE
//   payload:      scheme 0 stored bytes, 1 an LZ4 frame, 2 an LZ4 frame of the byte-grouped
//                 data (byte i of every 4-byte word gathered into group i % 4, groups concatenated)
// Decoding is single-pass with bounds checks on every read and write: a malformed or truncated
// range returns an error instead of touching memory outside the buffers.
#include <cstring>
#include <vector>

#include "omeio.h"

namespace {

constexpr size_t kChunkHeader = 8;
constexpr uint32_t kLz4FrameMagic = 0x184D2204u;

inline uint32_t rd24(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16); }
inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// one LZ4 block (sequences of literals + back-references) appended at dst[pos..]; `base` is the
// start of the window back-references may reach (linked frame blocks see earlier blocks)
int64_t lz4_block(const uint8_t* src, size_t len, uint8_t* dst, size_t cap, size_t pos, size_t base) {
  size_t i = 0;
  const size_t start = pos;
  while (i < len) {
    const uint8_t token = src[i++];
    size_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (i >= len) return -1;
        b = src[i++];
        lit += b;
      } while (b == 255);
    }
    if (lit > len - i || lit > cap - pos) return -2;
    memcpy(dst + pos, src + i, lit);
    i += lit;
    pos += lit;
    if (i == len) break;   // the last sequence has literals only
    if (len - i < 2) return -3;
    const size_t off = (size_t)src[i] | ((size_t)src[i + 1] << 8);
    i += 2;
    if (off == 0 || off > pos - base) return -4;
    size_t ml = (token & 15);
    if (ml == 15) {
      uint8_t b;
      do {
        if (i >= len) return -5;
        b = src[i++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (ml > cap - pos) return -6;
    const uint8_t* m = dst + pos - off;
    if (off >= ml) {
      memcpy(dst + pos, m, ml);
    } else {   // overlapping copy: repeats the last `off` bytes
      for (size_t k = 0; k < ml; ++k) dst[pos + k] = m[k];
    }
    pos += ml;
  }
  return (int64_t)(pos - start);
}

int64_t lz4_frame(const uint8_t* src, size_t len, uint8_t* dst, size_t cap) {
  if (len < 7 || rd32(src) != kLz4FrameMagic) return omeio_fail(-10, "lz4 frame: bad magic");
  const uint8_t flg = src[4];
  if ((flg >> 6) != 1) return omeio_fail(-11, "lz4 frame: unsupported version");
  const bool block_checksum = flg & 0x10, content_size = flg & 0x08, content_checksum = flg & 0x04,
             dict_id = flg & 0x01;
  size_t i = 6 + (content_size ? 8 : 0) + (dict_id ? 4 : 0) + 1;   // FLG BD [size] [dict] HC
  if (i > len) return omeio_fail(-12, "lz4 frame: truncated header");
  size_t pos = 0;
  for (;;) {
    if (len - i < 4) return omeio_fail(-13, "lz4 frame: truncated block size");
    const uint32_t bs = rd32(src + i);
    i += 4;
    if (bs == 0) break;   // end mark
    const size_t n = bs & 0x7FFFFFFFu;
    if (n > len - i) return omeio_fail(-14, "lz4 frame: truncated block");
    if (bs & 0x80000000u) {   // stored block
      if (n > cap - pos) return omeio_fail(-15, "lz4 frame: output overflow");
      memcpy(dst + pos, src + i, n);
      pos += n;
    } else {
      const int64_t w = lz4_block(src + i, n, dst, cap, pos, 0);
      if (w < 0) return omeio_fail(-16, "lz4 frame: corrupt block");
      pos += (size_t)w;
    }
    i += n + (block_checksum ? 4 : 0);
    if (i > len) return omeio_fail(-17, "lz4 frame: truncated block checksum");
  }
  if (content_checksum && len - i < 4) return omeio_fail(-18, "lz4 frame: truncated content checksum");
  return (int64_t)pos;
}

// inverse of the byte grouping: group g holds bytes g, g + 4, g + 8, ... of the original
void ungroup4(const uint8_t* g, size_t n, uint8_t* out) {
  const size_t q = n / 4, r = n % 4;
  size_t off[4], k = 0;
  for (int j = 0; j < 4; ++j) {
    off[j] = k;
    k += q + ((size_t)j < r ? 1 : 0);
  }
  for (size_t i = 0; i < n; ++i) out[i] = g[off[i % 4] + i / 4];
}

}  // namespace

OMEIO_API int64_t omeio_lz4_block_decode(const uint8_t* src, size_t len, uint8_t* dst, size_t cap) {
  const int64_t w = lz4_block(src, len, dst, cap, 0, 0);
  return w < 0 ? omeio_fail((int)w, "lz4 block: corrupt input") : w;
}

OMEIO_API int64_t omeio_lz4_frame_decode(const uint8_t* src, size_t len, uint8_t* dst, size_t cap) {
  return lz4_frame(src, len, dst, cap);
}

OMEIO_API int omeio_xet_scan(const uint8_t* src, size_t len, uint64_t* n_chunks, uint64_t* total) {
  size_t i = 0;
  uint64_t n = 0, t = 0;
  while (i < len) {
    if (len - i < kChunkHeader) return omeio_fail(-20, "xet: truncated chunk header");
    const uint8_t* h = src + i;
    if (h[0] != 0) return omeio_fail(-21, "xet: unknown chunk header version");
    const uint32_t clen = rd24(h + 1), scheme = h[4], ulen = rd24(h + 5);
    if (scheme > 2) return omeio_fail(-22, "xet: unknown compression scheme");
    if (scheme == 0 && clen != ulen) return omeio_fail(-23, "xet: stored chunk with mismatched lengths");
    if (clen > len - i - kChunkHeader) return omeio_fail(-24, "xet: truncated chunk payload");
    i += kChunkHeader + clen;
    ++n;
    t += ulen;
  }
  *n_chunks = n;
  *total = t;
  return 0;
}

OMEIO_API int64_t omeio_xet_decode(const uint8_t* src, size_t len, uint8_t* dst, size_t cap, uint64_t* offsets,
                                   uint64_t max_chunks) {
  size_t i = 0, pos = 0;
  uint64_t n = 0;
  std::vector<uint8_t> tmp;
  offsets[0] = 0;
  while (i < len) {
    if (n >= max_chunks) return omeio_fail(-30, "xet: more chunks than max_chunks");
    if (len - i < kChunkHeader) return omeio_fail(-20, "xet: truncated chunk header");
    const uint8_t* h = src + i;
    const uint32_t clen = rd24(h + 1), scheme = h[4], ulen = rd24(h + 5);
    if (clen > len - i - kChunkHeader) return omeio_fail(-24, "xet: truncated chunk payload");
    if (ulen > cap - pos) return omeio_fail(-31, "xet: output buffer too small");
    const uint8_t* p = h + kChunkHeader;
    if (scheme == 0) {
      if (clen != ulen) return omeio_fail(-23, "xet: stored chunk with mismatched lengths");
      memcpy(dst + pos, p, ulen);
    } else if (scheme == 1) {
      const int64_t w = lz4_frame(p, clen, dst + pos, ulen);
      if (w < 0) return w;
      if ((uint64_t)w != ulen) return omeio_fail(-32, "xet: LZ4 chunk decoded to the wrong length");
    } else if (scheme == 2) {
      tmp.resize(ulen);
      const int64_t w = lz4_frame(p, clen, tmp.data(), ulen);
      if (w < 0) return w;
      if ((uint64_t)w != ulen) return omeio_fail(-32, "xet: LZ4 chunk decoded to the wrong length");
      ungroup4(tmp.data(), ulen, dst + pos);
    } else {
      return omeio_fail(-22, "xet: unknown compression scheme");
    }
    pos += ulen;
    i += kChunkHeader + clen;
    offsets[++n] = pos;
  }
  return (int64_t)n;
}
