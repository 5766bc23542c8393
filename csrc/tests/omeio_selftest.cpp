// Host-side self test of libomeio, built with -fsanitize=address,undefined:
// safetensors header bounds checks, threaded ranged reads, parallel copy + MD5, AES-GCM file
// round trip and tamper detection.  No GPU needed (the device loader is covered by GPU tests).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../omeio/omeio.h"

#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, omeio_last_error()); \
      return 1;                                                   \
    }                                                             \
  } while (0)

static void write_file(const std::string& p, const std::vector<char>& d) {
  FILE* f = std::fopen(p.c_str(), "wb");
  std::fwrite(d.data(), 1, d.size(), f);
  std::fclose(f);
}

static std::vector<char> read_file(const std::string& p) {
  FILE* f = std::fopen(p.c_str(), "rb");
  std::vector<char> d;
  if (!f) return d;
  std::fseek(f, 0, SEEK_END);
  d.resize(std::ftell(f));
  std::fseek(f, 0, SEEK_SET);
  if (!d.empty() && std::fread(d.data(), 1, d.size(), f) != d.size()) d.clear();
  std::fclose(f);
  return d;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  // ---- safetensors header
  std::string hdr = "{\"w\":{\"dtype\":\"F32\",\"shape\":[2,2],\"data_offsets\":[0,16]}}";
  std::vector<char> st(8 + hdr.size() + 16, 0);
  uint64_t n = hdr.size();
  std::memcpy(st.data(), &n, 8);
  std::memcpy(st.data() + 8, hdr.data(), hdr.size());
  for (int i = 0; i < 16; ++i) st[8 + hdr.size() + i] = (char)i;
  write_file(dir + "/a.safetensors", st);
  char buf[4096];
  uint64_t hl = 0, off = 0;
  CHECK(omeio_st_header((dir + "/a.safetensors").c_str(), buf, sizeof buf, &hl, &off) == 0);
  CHECK(hl == hdr.size() && off == 8 + hdr.size() && std::string(buf) == hdr);
  CHECK(omeio_st_header((dir + "/a.safetensors").c_str(), buf, 8, &hl, &off) != 0);  // too small a buffer
  std::vector<char> bad = st;
  uint64_t huge = 1ull << 40;
  std::memcpy(bad.data(), &huge, 8);
  write_file(dir + "/bad.safetensors", bad);
  CHECK(omeio_st_header((dir + "/bad.safetensors").c_str(), buf, sizeof buf, &hl, &off) != 0);
  // ---- ranged reads (threads)
  std::vector<char> big(3 << 20);
  for (size_t i = 0; i < big.size(); ++i) big[i] = (char)(i * 131 + 7);
  write_file(dir + "/big.bin", big);
  std::vector<char> dst(big.size());
  uint64_t offs[3] = {0, 1 << 20, (2 << 20) + 5};
  uint64_t sizes[3] = {1 << 20, 1 << 20, (1 << 20) - 5};
  void* ptrs[3] = {dst.data(), dst.data() + (1 << 20), dst.data() + (2 << 20) + 5};
  CHECK(omeio_read_ranges((dir + "/big.bin").c_str(), 3, offs, sizes, ptrs, 4) == 0);
  CHECK(std::memcmp(dst.data(), big.data(), 2 << 20) == 0);
  CHECK(std::memcmp(dst.data() + (2 << 20) + 5, big.data() + (2 << 20) + 5, big.size() - (2 << 20) - 5) == 0);
  // ---- copy + md5
  char md5a[64], md5b[64];
  CHECK(omeio_copy_file((dir + "/big.bin").c_str(), (dir + "/big2.bin").c_str(), 4, md5a) == 0);
  CHECK(omeio_md5_file((dir + "/big.bin").c_str(), md5b) == 0);
  CHECK(std::strcmp(md5a, md5b) == 0 && read_file(dir + "/big2.bin") == big);
  // ---- AES-GCM
  uint8_t key[32], key2[32], nonce[12];
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1), key2[i] = (uint8_t)(i * 7 + 2);
  for (int i = 0; i < 12; ++i) nonce[i] = (uint8_t)i;
  CHECK(omeio_aes_gcm_encrypt_file((dir + "/big.bin").c_str(), (dir + "/big.enc").c_str(), key, nonce) == 0);
  CHECK(read_file(dir + "/big.enc").size() == big.size() + 28);
  CHECK(omeio_aes_gcm_decrypt_file((dir + "/big.enc").c_str(), (dir + "/big.dec").c_str(), key2) != 0);
  std::vector<char> enc = read_file(dir + "/big.enc");
  enc[100] ^= 1;
  write_file(dir + "/big.tampered", enc);
  CHECK(omeio_aes_gcm_decrypt_file((dir + "/big.tampered").c_str(), (dir + "/big.dec").c_str(), key) != 0);
  CHECK(omeio_aes_gcm_decrypt_file((dir + "/big.enc").c_str(), (dir + "/big.dec").c_str(), key) == 0);
  CHECK(read_file(dir + "/big.dec") == big);
  // Xet chunk runs: a valid run (stored chunk + LZ4-frame chunk with an overlapping match), then
  // thousands of random mutations / truncations that must fail cleanly, never read or write out
  // of bounds (this is network input)
  {
    std::vector<uint8_t> run;
    const char* stored = "stored-bytes";
    const uint32_t sl = (uint32_t)std::strlen(stored);
    uint8_t h0[8] = {0, (uint8_t)sl, 0, 0, 0, (uint8_t)sl, 0, 0};
    run.insert(run.end(), h0, h0 + 8);
    run.insert(run.end(), stored, stored + sl);
    // LZ4 frame: magic, FLG (v01 | independent), BD, HC, one block "ab" + match(off 2, len 10) + "!", end mark
    const uint8_t blk[] = {(2 << 4) | 6, 'a', 'b', 2, 0, 0x10, '!'};
    std::vector<uint8_t> fr = {0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0x00, (uint8_t)sizeof(blk), 0, 0, 0};
    fr.insert(fr.end(), blk, blk + sizeof(blk));
    fr.insert(fr.end(), {0, 0, 0, 0});
    uint8_t h1[8] = {0, (uint8_t)fr.size(), 0, 0, 1, 13, 0, 0};
    run.insert(run.end(), h1, h1 + 8);
    run.insert(run.end(), fr.begin(), fr.end());
    uint64_t n = 0, tot = 0;
    CHECK(omeio_xet_scan(run.data(), run.size(), &n, &tot) == 0 && n == 2 && tot == sl + 13);
    std::vector<uint8_t> out(tot);
    uint64_t offs[3];
    CHECK(omeio_xet_decode(run.data(), run.size(), out.data(), out.size(), offs, 2) == 2);
    CHECK(std::memcmp(out.data() + sl, "abababababab!", 13) == 0 && offs[2] == tot);
    unsigned seed = 12345;
    auto rnd = [&]() { return seed = seed * 1103515245u + 12345u; };
    for (int it = 0; it < 20000; ++it) {
      std::vector<uint8_t> m(run);
      const int flips = 1 + (int)(rnd() % 4);
      for (int f = 0; f < flips; ++f) m[rnd() % m.size()] = (uint8_t)rnd();
      m.resize(m.size() - (rnd() % 3 == 0 ? rnd() % m.size() : 0));
      std::vector<uint8_t> dst(64);
      uint64_t o[8];
      (void)omeio_xet_decode(m.data(), m.size(), dst.data(), dst.size(), o, 7);
      (void)omeio_lz4_block_decode(m.data(), m.size(), dst.data(), dst.size());
      (void)omeio_lz4_frame_decode(m.data(), m.size(), dst.data(), dst.size());
    }
  }
  std::printf("omeio selftest OK\n");
  return 0;
}
