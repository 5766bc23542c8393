// Native artifact I/O — see omeio.h.
#include "omeio.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>
#include <openssl/x509.h>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct Fd {
  int fd = -1;
  explicit Fd(int f) : fd(f) {}
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

std::atomic<uint64_t> g_bytes_read{0};   // bytes pread by this process (loader stats)

// pread the whole [off, off+len) range, retrying short reads.
bool pread_full(int fd, void* dst, uint64_t len, uint64_t off) {
  g_bytes_read.fetch_add(len, std::memory_order_relaxed);
  auto* p = static_cast<char*>(dst);
  while (len) {
    ssize_t r = pread(fd, p, std::min<uint64_t>(len, 1ull << 30), static_cast<off_t>(off));
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    if (r == 0) return false;
    p += r;
    off += static_cast<uint64_t>(r);
    len -= static_cast<uint64_t>(r);
  }
  return true;
}

bool pwrite_full(int fd, const void* src, uint64_t len, uint64_t off) {
  auto* p = static_cast<const char*>(src);
  while (len) {
    ssize_t r = pwrite(fd, p, std::min<uint64_t>(len, 1ull << 30), static_cast<off_t>(off));
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    off += static_cast<uint64_t>(r);
    len -= static_cast<uint64_t>(r);
  }
  return true;
}

// Read-only mapping of a file range for strided slice gathers.  A TP rank's slice of a
// row-parallel weight is a short piece (K / tp elements) of every row: one pread per row costs a
// syscall + page-cache lookup per few KB (2.6 GB/s measured for TP = 8, profiles/r04_llama70b_tp1.md),
// while a memcpy out of the mapping streams the same bytes at memory speed once the pages are
// resident (MADV_WILLNEED starts readahead of the whole range up front; ranks of one node share
// the page cache, so the file is read from storage once for all of them).
struct Mapping {
  void* base = MAP_FAILED;
  size_t len = 0;
  const char* at = nullptr;   // byte file_off of the request
  Mapping(int fd, uint64_t file_off, uint64_t span) {
    const uint64_t pg = static_cast<uint64_t>(sysconf(_SC_PAGESIZE));
    const uint64_t a = file_off / pg * pg;
    len = static_cast<size_t>(file_off - a + span);
    base = mmap(nullptr, len, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, static_cast<off_t>(a));
    if (base != MAP_FAILED) {
      madvise(base, len, MADV_WILLNEED);
      at = static_cast<const char*>(base) + (file_off - a);
    }
  }
  bool ok() const { return base != MAP_FAILED; }
  ~Mapping() {
    if (base != MAP_FAILED) munmap(base, len);
  }
};

// rows [r0, r0 + nr) of a strided slice from the mapping into a compact buffer
void gather_rows(const Mapping& m, uint64_t r0, uint64_t nr, uint64_t stride, uint64_t row_bytes, char* dst) {
  for (uint64_t r = 0; r < nr; ++r) memcpy(dst + r * row_bytes, m.at + (r0 + r) * stride, row_bytes);
  g_bytes_read.fetch_add(nr * row_bytes, std::memory_order_relaxed);
}

struct Piece {
  uint64_t file_off, len;
  char* dst;
};

std::vector<Piece> split(int n, const uint64_t* offs, const uint64_t* sizes, void* const* dsts, uint64_t chunk) {
  std::vector<Piece> out;
  for (int i = 0; i < n; ++i) {
    for (uint64_t o = 0; o < sizes[i]; o += chunk) {
      out.push_back({offs[i] + o, std::min(chunk, sizes[i] - o), static_cast<char*>(dsts[i]) + o});
    }
  }
  return out;
}

std::string hex(const unsigned char* d, unsigned n) {
  static const char* k = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (unsigned i = 0; i < n; ++i) {
    s[2 * i] = k[d[i] >> 4];
    s[2 * i + 1] = k[d[i] & 15];
  }
  return s;
}

}  // namespace

OMEIO_API const char* omeio_last_error() { return g_err.c_str(); }

// shared with the other translation units of the library (xet.cpp)
int omeio_fail(int code, const char* msg) { return fail(code, msg); }

OMEIO_API int omeio_st_header(const char* path, char* buf, size_t cap, uint64_t* header_len, uint64_t* data_offset) {
  Fd f(open(path, O_RDONLY | O_CLOEXEC));
  if (f.fd < 0) return fail(-ENOENT, std::string("open ") + path + ": " + strerror(errno));
  struct stat st {};
  fstat(f.fd, &st);
  uint64_t n = 0;
  if (!pread_full(f.fd, &n, 8, 0)) return fail(-EIO, "short read on safetensors length prefix");
  // Header is JSON; bound it (reference caps at 10 MB, we allow 100 MB for huge sharded MoE
  // headers) and against the file size so a corrupt prefix cannot trigger a giant allocation.
  if (n == 0 || n > (100ull << 20) || 8 + n > static_cast<uint64_t>(st.st_size))
    return fail(-EINVAL, "invalid safetensors header length " + std::to_string(n));
  *header_len = n;
  *data_offset = 8 + n;
  if (cap < n + 1) return fail(-ENOSPC, "buffer too small");
  if (!pread_full(f.fd, buf, n, 8)) return fail(-EIO, "short read on safetensors header");
  buf[n] = 0;
  if (buf[0] != '{') return fail(-EINVAL, "safetensors header is not a JSON object");
  return 0;
}

OMEIO_API int omeio_read_ranges(const char* path, int n, const uint64_t* offs, const uint64_t* sizes,
                                void* const* dst, int nthreads) {
  Fd f(open(path, O_RDONLY | O_CLOEXEC));
  if (f.fd < 0) return fail(-ENOENT, std::string("open ") + path + ": " + strerror(errno));
  posix_fadvise(f.fd, 0, 0, POSIX_FADV_SEQUENTIAL);
  auto pieces = split(n, offs, sizes, dst, 64ull << 20);
  nthreads = std::max(1, std::min<int>(nthreads, static_cast<int>(pieces.size())));
  std::atomic<int> err{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&, t] {
      size_t lo = pieces.size() * t / nthreads, hi = pieces.size() * (t + 1) / nthreads;
      for (size_t i = lo; i < hi && !err.load(); ++i)
        if (!pread_full(f.fd, pieces[i].dst, pieces[i].len, pieces[i].file_off)) err = -EIO;
    });
  }
  for (auto& x : th) x.join();
  return err ? fail(err, std::string("read failed: ") + path) : 0;
}

OMEIO_API int omeio_load_ranges(const char* path, int n, const uint64_t* offs, const uint64_t* sizes,
                                void* const* dst, void* stream, int nthreads, uint64_t chunk) {
  Fd f(open(path, O_RDONLY | O_CLOEXEC));
  if (f.fd < 0) return fail(-ENOENT, std::string("open ") + path + ": " + strerror(errno));
  posix_fadvise(f.fd, 0, 0, POSIX_FADV_SEQUENTIAL);
  if (chunk == 0) chunk = 16ull << 20;
  // Make sure the caller's pending work on the destination (e.g. allocation-side memsets) is done.
  if (hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess) return fail(-EIO, "stream sync failed");
  auto pieces = split(n, offs, sizes, dst, chunk);
  if (pieces.empty()) return 0;
  nthreads = std::max(1, std::min<int>(nthreads, static_cast<int>(pieces.size())));
  std::atomic<int> err{0};
  std::string msg;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&, t] {
      hipStream_t s;
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        err = -EIO;
        return;
      }
      void* stage[2] = {nullptr, nullptr};
      hipEvent_t ev[2];
      bool used[2] = {false, false};
      for (int b = 0; b < 2; ++b) {
        if (hipHostMalloc(&stage[b], chunk, hipHostMallocDefault) != hipSuccess) err = -ENOMEM;
        hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
      }
      size_t lo = pieces.size() * t / nthreads, hi = pieces.size() * (t + 1) / nthreads;
      int b = 0;
      for (size_t i = lo; i < hi && !err.load(); ++i, b ^= 1) {
        if (used[b] && hipEventSynchronize(ev[b]) != hipSuccess) {
          err = -EIO;
          break;
        }
        if (!pread_full(f.fd, stage[b], pieces[i].len, pieces[i].file_off)) {
          err = -EIO;
          break;
        }
        if (hipMemcpyAsync(pieces[i].dst, stage[b], pieces[i].len, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipEventRecord(ev[b], s) != hipSuccess) {
          err = -EIO;
          break;
        }
        used[b] = true;
      }
      hipStreamSynchronize(s);
      for (int k = 0; k < 2; ++k) {
        if (stage[k]) hipHostFree(stage[k]);
        hipEventDestroy(ev[k]);
      }
      hipStreamDestroy(s);
    });
  }
  for (auto& x : th) x.join();
  return err ? fail(err, std::string("device load failed: ") + path) : 0;
}

// Column shard of a row-major [nrows][*] tensor: nrows slices of row_bytes at
// file_off + r * file_stride, packed contiguously into dst (the [nrows][row_bytes] shard of a
// row-parallel TP weight).  Only the slices are read and only they reach HBM: each thread
// preads a run of rows into its pinned stage (one pread per row) and sends the packed run with
// ONE hipMemcpyAsync, double-buffered.
OMEIO_API int omeio_load_strided(const char* path, uint64_t file_off, uint64_t nrows, uint64_t file_stride,
                                 uint64_t row_bytes, void* dst, void* stream, int nthreads, uint64_t chunk) {
  if (nrows == 0 || row_bytes == 0) return 0;
  Fd f(open(path, O_RDONLY | O_CLOEXEC));
  if (f.fd < 0) return fail(-ENOENT, std::string("open ") + path + ": " + strerror(errno));
  if (chunk == 0) chunk = 16ull << 20;
  if (hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess) return fail(-EIO, "stream sync failed");
  const uint64_t rows_per = std::max<uint64_t>(1, chunk / row_bytes);
  const uint64_t nruns = (nrows + rows_per - 1) / rows_per;
  const uint64_t stage_bytes = rows_per * row_bytes;
  const Mapping map(f.fd, file_off, (nrows - 1) * file_stride + row_bytes);   // pread per row if it fails
  nthreads = std::max(1, std::min<int>(nthreads, static_cast<int>(nruns)));
  std::atomic<int> err{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&, t] {
      hipStream_t s;
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        err = -EIO;
        return;
      }
      void* stage[2] = {nullptr, nullptr};
      hipEvent_t ev[2];
      bool used[2] = {false, false};
      for (int b = 0; b < 2; ++b) {
        if (hipHostMalloc(&stage[b], stage_bytes, hipHostMallocDefault) != hipSuccess) err = -ENOMEM;
        hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
      }
      const uint64_t lo = nruns * t / nthreads, hi = nruns * (t + 1) / nthreads;
      int b = 0;
      for (uint64_t run = lo; run < hi && !err.load(); ++run, b ^= 1) {
        if (used[b] && hipEventSynchronize(ev[b]) != hipSuccess) {
          err = -EIO;
          break;
        }
        const uint64_t r0 = run * rows_per, nr = std::min(rows_per, nrows - r0);
        char* st = static_cast<char*>(stage[b]);
        if (map.ok()) {
          gather_rows(map, r0, nr, file_stride, row_bytes, st);
        } else {
          for (uint64_t r = 0; r < nr; ++r)
            if (!pread_full(f.fd, st + r * row_bytes, row_bytes, file_off + (r0 + r) * file_stride)) {
              err = -EIO;
              break;
            }
        }
        if (err.load()) break;
        if (hipMemcpyAsync(static_cast<char*>(dst) + r0 * row_bytes, st, nr * row_bytes, hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipEventRecord(ev[b], s) != hipSuccess) {
          err = -EIO;
          break;
        }
        used[b] = true;
      }
      hipStreamSynchronize(s);
      for (int k = 0; k < 2; ++k) {
        if (stage[k]) hipHostFree(stage[k]);
        hipEventDestroy(ev[k]);
      }
      hipStreamDestroy(s);
    });
  }
  for (auto& x : th) x.join();
  return err ? fail(err, std::string("strided device load failed: ") + path) : 0;
}

// host-memory form of omeio_load_strided (CPU loads and tests)
OMEIO_API int omeio_read_strided(const char* path, uint64_t file_off, uint64_t nrows, uint64_t file_stride,
                                 uint64_t row_bytes, void* dst) {
  Fd f(open(path, O_RDONLY | O_CLOEXEC));
  if (f.fd < 0) return fail(-ENOENT, std::string("open ") + path + ": " + strerror(errno));
  if (nrows == 0 || row_bytes == 0) return 0;
  const Mapping map(f.fd, file_off, (nrows - 1) * file_stride + row_bytes);
  if (map.ok()) {   // gather from the mapping, a few threads over row ranges
    const int nt = static_cast<int>(std::min<uint64_t>(8, std::max<uint64_t>(1, nrows * row_bytes >> 20)));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        const uint64_t lo = nrows * t / nt, hi = nrows * (t + 1) / nt;
        gather_rows(map, lo, hi - lo, file_stride, row_bytes, static_cast<char*>(dst) + lo * row_bytes);
      });
    for (auto& x : th) x.join();
    return 0;
  }
  for (uint64_t r = 0; r < nrows; ++r)
    if (!pread_full(f.fd, static_cast<char*>(dst) + r * row_bytes, row_bytes, file_off + r * file_stride))
      return fail(-EIO, std::string("strided read failed: ") + path);
  return 0;
}

OMEIO_API uint64_t omeio_bytes_read() { return g_bytes_read.load(); }

OMEIO_API int omeio_md5_file(const char* path, char* md5_hex) {
  Fd f(open(path, O_RDONLY | O_CLOEXEC));
  if (f.fd < 0) return fail(-ENOENT, std::string("open ") + path + ": " + strerror(errno));
  posix_fadvise(f.fd, 0, 0, POSIX_FADV_SEQUENTIAL);
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  EVP_DigestInit_ex(ctx, EVP_md5(), nullptr);
  std::vector<char> buf(8 << 20);
  ssize_t r;
  while ((r = read(f.fd, buf.data(), buf.size())) > 0) EVP_DigestUpdate(ctx, buf.data(), static_cast<size_t>(r));
  unsigned char d[EVP_MAX_MD_SIZE];
  unsigned dl = 0;
  EVP_DigestFinal_ex(ctx, d, &dl);
  EVP_MD_CTX_free(ctx);
  if (r < 0) return fail(-EIO, "read failed");
  std::string h = hex(d, dl);
  memcpy(md5_hex, h.c_str(), h.size() + 1);
  return 0;
}

OMEIO_API int omeio_copy_file(const char* src, const char* dst, int nthreads, char* md5_hex) {
  Fd in(open(src, O_RDONLY | O_CLOEXEC));
  if (in.fd < 0) return fail(-ENOENT, std::string("open ") + src + ": " + strerror(errno));
  struct stat st {};
  fstat(in.fd, &st);
  Fd out(open(dst, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644));
  if (out.fd < 0) return fail(-EACCES, std::string("create ") + dst + ": " + strerror(errno));
  const uint64_t size = static_cast<uint64_t>(st.st_size);
  if (size && ftruncate(out.fd, static_cast<off_t>(size)) != 0) return fail(-EIO, "ftruncate failed");
  const uint64_t chunk = 32ull << 20;
  const uint64_t nchunks = (size + chunk - 1) / chunk;
  nthreads = std::max(1, std::min<int>(nthreads, static_cast<int>(std::max<uint64_t>(1, nchunks))));
  std::atomic<uint64_t> next{0};
  std::atomic<int> err{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&] {
      std::vector<char> buf(chunk);
      for (uint64_t c; (c = next.fetch_add(1)) < nchunks && !err.load();) {
        uint64_t off = c * chunk, len = std::min(chunk, size - off);
        if (!pread_full(in.fd, buf.data(), len, off) || !pwrite_full(out.fd, buf.data(), len, off)) err = -EIO;
      }
    });
  }
  for (auto& x : th) x.join();
  if (err) return fail(err, std::string("copy failed: ") + src + " -> " + dst);
  if (md5_hex) return omeio_md5_file(dst, md5_hex);
  return 0;
}

OMEIO_API int omeio_aes_gcm_encrypt(const uint8_t* in, size_t in_len, const uint8_t* key, const uint8_t* nonce,
                                    uint8_t* out, size_t* out_len) {
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  int ok = EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), nullptr, nullptr, nullptr) &&
           EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 12, nullptr) &&
           EVP_EncryptInit_ex(c, nullptr, nullptr, key, nonce);
  memcpy(out, nonce, 12);
  int l1 = 0, l2 = 0;
  ok = ok && EVP_EncryptUpdate(c, out + 12, &l1, in, static_cast<int>(in_len)) &&
       EVP_EncryptFinal_ex(c, out + 12 + l1, &l2) &&
       EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, out + 12 + l1 + l2);
  EVP_CIPHER_CTX_free(c);
  if (!ok) return fail(-EINVAL, "AES-GCM encrypt failed");
  *out_len = 12 + static_cast<size_t>(l1 + l2) + 16;
  return 0;
}

OMEIO_API int omeio_aes_gcm_decrypt(const uint8_t* in, size_t in_len, const uint8_t* key, uint8_t* out,
                                    size_t* out_len) {
  if (in_len < 28) return fail(-EINVAL, "ciphertext too short");
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  int l1 = 0, l2 = 0;
  int ok = EVP_DecryptInit_ex(c, EVP_aes_256_gcm(), nullptr, nullptr, nullptr) &&
           EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 12, nullptr) &&
           EVP_DecryptInit_ex(c, nullptr, nullptr, key, in) &&
           EVP_DecryptUpdate(c, out, &l1, in + 12, static_cast<int>(in_len - 28)) &&
           EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, const_cast<uint8_t*>(in + in_len - 16));
  ok = ok && EVP_DecryptFinal_ex(c, out + l1, &l2) > 0;
  EVP_CIPHER_CTX_free(c);
  if (!ok) return fail(-EBADMSG, "AES-GCM authentication failed");
  *out_len = static_cast<size_t>(l1 + l2);
  return 0;
}

namespace {
int gcm_file(const char* src, const char* dst, const uint8_t* key, const uint8_t* nonce_or_null, bool enc) {
  Fd in(open(src, O_RDONLY | O_CLOEXEC));
  if (in.fd < 0) return fail(-ENOENT, std::string("open ") + src + ": " + strerror(errno));
  struct stat st {};
  fstat(in.fd, &st);
  const uint64_t size = static_cast<uint64_t>(st.st_size);
  uint8_t nonce[12], tag[16];
  uint64_t body_off = 0, body_len = size;
  if (enc) {
    memcpy(nonce, nonce_or_null, 12);
  } else {
    if (size < 28) return fail(-EINVAL, "encrypted file too short");
    if (!pread_full(in.fd, nonce, 12, 0) || !pread_full(in.fd, tag, 16, size - 16)) return fail(-EIO, "read failed");
    body_off = 12;
    body_len = size - 28;
  }
  std::string tmp = std::string(dst) + ".omeio-tmp";
  Fd out(open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644));
  if (out.fd < 0) return fail(-EACCES, "create " + tmp + ": " + strerror(errno));
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  int ok = (enc ? EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), nullptr, nullptr, nullptr)
                : EVP_DecryptInit_ex(c, EVP_aes_256_gcm(), nullptr, nullptr, nullptr)) &&
           EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 12, nullptr) &&
           (enc ? EVP_EncryptInit_ex(c, nullptr, nullptr, key, nonce) : EVP_DecryptInit_ex(c, nullptr, nullptr, key, nonce));
  uint64_t woff = 0;
  if (ok && enc) ok = pwrite_full(out.fd, nonce, 12, 0), woff = 12;
  const uint64_t chunk = 8ull << 20;
  std::vector<uint8_t> ib(chunk), ob(chunk + 32);
  for (uint64_t o = 0; ok && o < body_len; o += chunk) {
    uint64_t len = std::min(chunk, body_len - o);
    int ol = 0;
    ok = pread_full(in.fd, ib.data(), len, body_off + o) &&
         (enc ? EVP_EncryptUpdate(c, ob.data(), &ol, ib.data(), static_cast<int>(len))
              : EVP_DecryptUpdate(c, ob.data(), &ol, ib.data(), static_cast<int>(len))) &&
         pwrite_full(out.fd, ob.data(), static_cast<uint64_t>(ol), woff);
    woff += static_cast<uint64_t>(ol);
  }
  int fl = 0;
  if (ok) {
    if (enc) {
      ok = EVP_EncryptFinal_ex(c, ob.data(), &fl) && pwrite_full(out.fd, ob.data(), fl, woff) &&
           EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, tag) && pwrite_full(out.fd, tag, 16, woff + fl);
    } else {
      ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, tag) && EVP_DecryptFinal_ex(c, ob.data(), &fl) > 0 &&
           pwrite_full(out.fd, ob.data(), fl, woff);
    }
  }
  EVP_CIPHER_CTX_free(c);
  if (!ok) {
    unlink(tmp.c_str());
    return fail(-EBADMSG, enc ? "AES-GCM encryption failed" : "AES-GCM authentication failed (wrong key or corrupt file)");
  }
  if (rename(tmp.c_str(), dst) != 0) return fail(-EIO, std::string("rename failed: ") + strerror(errno));
  return 0;
}
}  // namespace

OMEIO_API int omeio_aes_gcm_encrypt_file(const char* src, const char* dst, const uint8_t* key, const uint8_t* nonce) {
  return gcm_file(src, dst, key, nonce, true);
}

OMEIO_API int omeio_aes_gcm_decrypt_file(const char* src, const char* dst, const uint8_t* key) {
  return gcm_file(src, dst, key, nullptr, false);
}

// ------------------------------------------------------------------------------------------
// RSA PKCS#1 v1.5 / SHA-256 signatures for the cloud request signers (OCI API keys, GCP service
// accounts) through OpenSSL: the private-key operation uses OpenSSL's blinded constant-time RSA
// (CRT), and verification checks the complete DigestInfo encoding.  The key is a PEM (PKCS#1 or
// PKCS#8 private key; for verification also a public key / SubjectPublicKeyInfo).
// ------------------------------------------------------------------------------------------
namespace {
EVP_PKEY* pem_key(const char* pem, size_t n, bool want_private) {
  BIO* b = BIO_new_mem_buf(pem, static_cast<int>(n));
  if (!b) return nullptr;
  EVP_PKEY* k = PEM_read_bio_PrivateKey(b, nullptr, nullptr, const_cast<char*>(""));
  if (!k && !want_private) {
    BIO_reset(b);
    k = PEM_read_bio_PUBKEY(b, nullptr, nullptr, nullptr);
  }
  BIO_free(b);
  if (k && EVP_PKEY_base_id(k) != EVP_PKEY_RSA) {
    EVP_PKEY_free(k);
    return nullptr;
  }
  return k;
}
}  // namespace

// sig: capacity *sig_len bytes (>= the modulus size); *sig_len receives the signature length
OMEIO_API int omeio_rsa_sign_sha256(const char* pem, size_t pem_len, const uint8_t* msg, size_t n, uint8_t* sig,
                                    size_t* sig_len) {
  EVP_PKEY* k = pem_key(pem, pem_len, true);
  if (!k) return fail(-EINVAL, "not an RSA private key (or an encrypted one)");
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  int rc = -EIO;
  size_t need = 0;
  if (c && EVP_DigestSignInit(c, nullptr, EVP_sha256(), nullptr, k) == 1 && EVP_DigestSignUpdate(c, msg, n) == 1 &&
      EVP_DigestSignFinal(c, nullptr, &need) == 1) {
    if (need > *sig_len) {
      rc = fail(-ENOSPC, "signature buffer too small");
    } else if (EVP_DigestSignFinal(c, sig, sig_len) == 1) {
      rc = 0;
    }
  }
  if (rc == -EIO) rc = fail(-EIO, "RSA signing failed");
  EVP_MD_CTX_free(c);
  EVP_PKEY_free(k);
  return rc;
}

// 1 = valid, 0 = invalid signature, < 0 = bad key
OMEIO_API int omeio_rsa_verify_sha256(const char* pem, size_t pem_len, const uint8_t* msg, size_t n,
                                      const uint8_t* sig, size_t sig_len) {
  EVP_PKEY* k = pem_key(pem, pem_len, false);
  if (!k) return fail(-EINVAL, "not an RSA key");
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  int ok = 0;
  if (c && EVP_DigestVerifyInit(c, nullptr, EVP_sha256(), nullptr, k) == 1 && EVP_DigestVerifyUpdate(c, msg, n) == 1)
    ok = EVP_DigestVerifyFinal(c, sig, sig_len) == 1 ? 1 : 0;
  EVP_MD_CTX_free(c);
  EVP_PKEY_free(k);
  return ok;
}

namespace {
int bio_to(BIO* b, char* out, size_t cap) {
  char* p = nullptr;
  const long n = BIO_get_mem_data(b, &p);
  if (n < 0 || static_cast<size_t>(n) + 1 > cap) return fail(-ENOSPC, "output buffer too small");
  memcpy(out, p, static_cast<size_t>(n));
  out[n] = 0;
  return 0;
}
}  // namespace

// Fresh RSA key pair (OCI instance-principal session keys): PKCS#8 private PEM + SPKI public PEM.
OMEIO_API int omeio_rsa_keygen(int bits, char* priv_pem, size_t priv_cap, char* pub_pem, size_t pub_cap) {
  EVP_PKEY_CTX* c = EVP_PKEY_CTX_new_id(EVP_PKEY_RSA, nullptr);
  EVP_PKEY* k = nullptr;
  int rc = -EIO;
  if (c && EVP_PKEY_keygen_init(c) == 1 && EVP_PKEY_CTX_set_rsa_keygen_bits(c, bits) == 1 &&
      EVP_PKEY_keygen(c, &k) == 1) {
    BIO* a = BIO_new(BIO_s_mem());
    BIO* b = BIO_new(BIO_s_mem());
    if (a && b && PEM_write_bio_PrivateKey(a, k, nullptr, nullptr, 0, nullptr, nullptr) == 1 &&
        PEM_write_bio_PUBKEY(b, k) == 1) {
      rc = bio_to(a, priv_pem, priv_cap);
      if (rc == 0) rc = bio_to(b, pub_pem, pub_cap);
    }
    BIO_free(a);
    BIO_free(b);
  }
  if (rc == -EIO) rc = fail(-EIO, "RSA key generation failed");
  EVP_PKEY_free(k);
  EVP_PKEY_CTX_free(c);
  return rc;
}

// X.509 certificate facts for request signing: the one-line RFC 2253 subject, and the SHA-1 /
// SHA-256 fingerprints of the DER encoding as colon-separated upper-case hex.
OMEIO_API int omeio_x509_info(const char* pem, size_t n, char* subject, size_t subject_cap, char* sha1_fp,
                              char* sha256_fp) {
  BIO* in = BIO_new_mem_buf(pem, static_cast<int>(n));
  X509* x = in ? PEM_read_bio_X509(in, nullptr, nullptr, nullptr) : nullptr;
  BIO_free(in);
  if (!x) return fail(-EINVAL, "not a PEM X.509 certificate");
  int rc = 0;
  BIO* b = BIO_new(BIO_s_mem());
  if (!b || X509_NAME_print_ex(b, X509_get_subject_name(x), 0, XN_FLAG_RFC2253) < 0) rc = fail(-EIO, "subject");
  if (rc == 0) rc = bio_to(b, subject, subject_cap);
  BIO_free(b);
  const EVP_MD* mds[2] = {EVP_sha1(), EVP_sha256()};
  char* outs[2] = {sha1_fp, sha256_fp};
  for (int i = 0; i < 2 && rc == 0; ++i) {
    unsigned char md[EVP_MAX_MD_SIZE];
    unsigned int len = 0;
    if (X509_digest(x, mds[i], md, &len) != 1) {
      rc = fail(-EIO, "certificate digest failed");
      break;
    }
    static const char* hx = "0123456789ABCDEF";
    char* o = outs[i];
    for (unsigned int j = 0; j < len; ++j) {
      if (j) *o++ = ':';
      *o++ = hx[md[j] >> 4];
      *o++ = hx[md[j] & 15];
    }
    *o = 0;
  }
  X509_free(x);
  return rc;
}
