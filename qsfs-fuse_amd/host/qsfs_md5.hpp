// qsfs-fuse_amd/host/qsfs_md5.hpp -- C++ drop-in for qsfs's src/base/MD5.h.
//
// Header-only layer over the C-ABI (include/qsmd5.h) that keeps the
// reference's interface so QSClient compiles unchanged apart from the include:
//
//   std::string md5(const std::string)                 MD5.h:95, MD5.cpp:335-339
//   std::string md5(const shared_ptr<std::iostream>&)  MD5.h:96, MD5.cpp:341-349
//   class MD5 { update; finalize; hexdigest; << }      MD5.h:51-93
//
// plus the batch forms the reference lacks: md5_batch() and md5_file_parts()
// (all parts of a file in one GPU pass).
//
// md5(stream) hashes exactly the bytes the reference hashes -- from position 0
// to the end of the stream's get area, i.e. the first lengthToRead bytes of a
// qsfs StreamBuf (StreamBuf.cpp:32-48) -- and, like the reference, leaves the
// read position at 0 (MD5.cpp:343, 346).  Unlike the reference it does not
// copy the buffer twice through a stringstream (MD5.cpp:342-345): when the
// stream buffer exposes its whole content as the get area (StreamBuf does),
// the bytes are handed to the GPU in place.
//
// Failure: the reference could only throw std::bad_alloc.  A GPU failure here
// throws qsmd5::Error (a std::runtime_error) -- a Content-MD5 must never
// silently become "".
//
// The stream overload is a template over the smart-pointer type, so it accepts
// boost::shared_ptr<std::iostream> (what qsfs passes) and std::shared_ptr alike.
#ifndef QSFS_AMD_QSFS_MD5_HPP_
#define QSFS_AMD_QSFS_MD5_HPP_

#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/qsmd5.h"

namespace qsmd5 {

class Error : public std::runtime_error {
 public:
  Error(int code, const char* what)
      : std::runtime_error(std::string(what) + ": " + qsmd5_strerror(code) + " (" +
                           qsmd5_last_error() + ")"),
        code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

namespace detail {

// Access to the protected get-area pointers of any std::streambuf.
struct GetArea : std::streambuf {
  using std::streambuf::eback;
  using std::streambuf::egptr;
  using std::streambuf::gptr;
};

inline std::string hex(const uint8_t d[16]) {
  char b[33];
  qsmd5_hex(d, b);
  return std::string(b, 32);
}

inline void check(int rc, const char* what) {
  if (rc != 0) throw Error(rc, what);
}

}  // namespace detail

// MD5 of [p, p + len) as 32 lowercase hex characters.
inline std::string md5_bytes(const void* p, uint64_t len) {
  uint8_t d[16];
  detail::check(qsmd5_hash_one(p, len, d), "qsmd5_hash_one");
  return detail::hex(d);
}

// md5(const std::string) -- MD5.cpp:335-339.
inline std::string md5(const std::string& str) { return md5_bytes(str.data(), str.size()); }

namespace detail {
// Enabled for anything with ->seekg / ->rdbuf (boost/std shared_ptr<iostream>).
template <class P>
using if_stream_ptr = decltype(std::declval<const P&>()->rdbuf(),
                               std::declval<const P&>()->seekg(0, std::ios_base::beg), 0);
}  // namespace detail

// md5(const shared_ptr<iostream>&) -- MD5.cpp:341-349.
template <class StreamPtr, detail::if_stream_ptr<StreamPtr> = 0>
std::string md5(const StreamPtr& stream) {
  stream->seekg(0, std::ios_base::beg);
  // The read position is back at 0 however this returns (MD5.cpp:346), a
  // hashing failure's exception included.
  struct Rewind {
    const StreamPtr& s;
    ~Rewind() {
      try {  // a stream with exceptions() set must not throw out of here
        s->clear();
        s->seekg(0, std::ios_base::beg);
      } catch (...) {
      }
    }
  } rewind{stream};
  std::streambuf* sb = stream->rdbuf();
  std::string out;
  if (sb) {
    char* (std::streambuf::*p_gptr)() const = &detail::GetArea::gptr;
    char* (std::streambuf::*p_egptr)() const = &detail::GetArea::egptr;
    // Zero-copy only when the get area is the whole remaining content.
    const std::streamoff end = sb->pubseekoff(0, std::ios_base::end, std::ios_base::in);
    sb->pubseekoff(0, std::ios_base::beg, std::ios_base::in);
    const char* g = (sb->*p_gptr)();
    const char* e = (sb->*p_egptr)();
    if (g && e >= g && end >= 0 && std::streamoff(e - g) == end) {
      out = md5_bytes(g, static_cast<uint64_t>(e - g));
    } else {
      std::vector<char> buf;
      char tmp[1 << 16];
      std::streamsize got;
      while ((got = sb->sgetn(tmp, sizeof tmp)) > 0) buf.insert(buf.end(), tmp, tmp + got);
      out = md5_bytes(buf.data(), buf.size());
    }
  } else {
    out = md5_bytes(nullptr, 0);
  }
  return out;
}

// Batch form: the hex MD5 of every buffer, in order,
// from ONE qsmd5_hash_batch call -- one GPU pass for all parts of a file
// instead of one md5(buffer) per part (File.cpp:641,644 hash them serially).
inline std::vector<std::string> md5_batch(const std::vector<qsmd5_chunk>& chunks) {
  std::vector<std::string> out;
  if (chunks.empty()) return out;
  std::vector<uint8_t> dig(16 * chunks.size());
  detail::check(qsmd5_hash_batch(chunks.data(), chunks.size(),
                                 reinterpret_cast<uint8_t(*)[16]>(dig.data())),
                "qsmd5_hash_batch");
  out.reserve(chunks.size());
  for (size_t i = 0; i < chunks.size(); ++i) out.push_back(detail::hex(&dig[16 * i]));
  return out;
}

// One upload part and its Content-MD5 text.
struct PartMD5 {
  qsmd5_part part;  // number, offset, size as QSTransferManager::PrepareUpload slices
  std::string md5;  // what UploadMultipart would pass to SetContentMD5 (QSClient.cpp:370)
};

// Every part of a file held in one buffer, sliced exactly as PrepareUpload
// does (QSTransferManager.cpp:475-550: single PutObject below `threshold`,
// else `buf_size` parts with the short tail averaged into the previous part
// when it is below `min_part`), hashed in one batch.  Defaults are qsfs's:
// -b 10 MiB buffers, 4 MiB minimum part, 20 MiB multipart threshold.
inline std::vector<PartMD5> md5_file_parts(const void* file, uint64_t size,
                                           uint64_t buf_size = 10ull << 20,
                                           uint64_t min_part = 4ull << 20,
                                           uint64_t threshold = 20ull << 20) {
  size_t n = 0;
  detail::check(qsmd5_plan_parts(size, buf_size, min_part, threshold, 0, nullptr, 0, &n),
                "qsmd5_plan_parts");
  std::vector<qsmd5_part> parts(n);
  detail::check(qsmd5_plan_parts(size, buf_size, min_part, threshold, 0, parts.data(), n, &n),
                "qsmd5_plan_parts");
  std::vector<uint8_t> dig(16 * n);
  detail::check(qsmd5_hash_parts(file, parts.data(), n, reinterpret_cast<uint8_t(*)[16]>(dig.data())),
                "qsmd5_hash_parts");
  std::vector<PartMD5> out(n);
  for (size_t i = 0; i < n; ++i) out[i] = PartMD5{parts[i], detail::hex(&dig[16 * i])};
  return out;
}

// Download-side integrity check: true if the MD5 of
// [p, p+len) equals a single-part object's ETag (QSClient.cpp:321-323).
// Throws qsmd5::Error for a multipart/malformed ETag or a GPU failure.
inline bool verify_etag(const void* p, uint64_t len, const std::string& etag) {
  const int rc = qsmd5_verify_etag(p, len, etag.c_str());
  if (rc < 0) throw Error(rc, "qsmd5_verify_etag");
  return rc == 1;
}

// RFC 1864 Content-MD5 header value (base64 of the raw digest) from the
// 32-char hex text md5() returns.  Throws on bad hex.
inline std::string content_md5_from_hex(const std::string& hex) {
  if (hex.size() != 32) throw Error(-22, "content_md5_from_hex: need 32 hex chars");
  uint8_t d[16];
  for (int i = 0; i < 32; ++i) {
    const char c = hex[i];
    const int v = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10
                : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
    if (v < 0) throw Error(-22, "content_md5_from_hex: not hex");
    d[i / 2] = (uint8_t)(i % 2 ? (d[i / 2] | v) : v << 4);
  }
  char b[25];
  qsmd5_base64(d, b);
  return std::string(b, 24);
}

// The runtime's lifetime for a daemon's main() or FUSE init/destroy pair
// (INTEGRATION.md §2): initialises the GPU runtime up front (after the fork
// fuse_main does, Operations.cpp:1520-1549) and releases it with
// qsmd5_shutdown() before static destructors run.  init() reports failure as
// its return code; without a GPU the calls still hash on the CPU under the
// default routing.  Stop every hashing thread and destroy every MD5 object
// before the guard goes out of scope.
class Runtime {
 public:
  Runtime() : init_rc_(qsmd5_init(0)) {}
  Runtime(const Runtime&) = delete;
  Runtime& operator=(const Runtime&) = delete;
  ~Runtime() { (void)qsmd5_shutdown(); }
  int init_rc() const { return init_rc_; }

 private:
  int init_rc_;
};

// class MD5 -- MD5.h:51-93, over the streaming C-ABI context.
class MD5 {
 public:
  typedef unsigned int size_type;  // as the reference (MD5.h:53)

  MD5() { detail::check(qsmd5_ctx_create(&ctx_), "qsmd5_ctx_create"); }
  explicit MD5(const std::string& text) : MD5() {
    update(text.c_str(), static_cast<size_type>(text.length()));
    finalize();
  }
  // A value type, as the reference's (implicit copy members; operator<< takes
  // it by value, MD5.h:61): a copy carries the running state and then hashes
  // on by itself (qsmd5_ctx_copy).
  MD5(const MD5& o) : finalized_(o.finalized_) {
    std::memcpy(digest_, o.digest_, 16);
    if (o.ctx_) detail::check(qsmd5_ctx_copy(o.ctx_, &ctx_), "qsmd5_ctx_copy");
  }
  MD5& operator=(const MD5& o) {
    if (this != &o) {
      MD5 tmp(o);
      swap(tmp);
    }
    return *this;
  }
  MD5(MD5&& o) noexcept : ctx_(o.ctx_), finalized_(o.finalized_) {
    std::memcpy(digest_, o.digest_, 16);
    o.ctx_ = nullptr;
  }
  MD5& operator=(MD5&& o) noexcept {
    swap(o);
    return *this;
  }
  ~MD5() { qsmd5_ctx_destroy(ctx_); }
  void swap(MD5& o) noexcept {
    std::swap(ctx_, o.ctx_);
    std::swap(finalized_, o.finalized_);
    uint8_t t[16];
    std::memcpy(t, digest_, 16);
    std::memcpy(digest_, o.digest_, 16);
    std::memcpy(o.digest_, t, 16);
  }

  // After finalize() the reference's update() folds the bytes into a state
  // nobody reads again (finalize zeroised the count, MD5.cpp:306-309, and
  // never runs twice): the digest and hexdigest() stay as they were.  The
  // drop-in does the same -- a no-op -- rather than throw.
  void update(const unsigned char* buf, size_type length) {
    if (finalized_) return;
    detail::check(qsmd5_ctx_update(ctx_, buf, length), "qsmd5_ctx_update");
  }
  void update(const char* buf, size_type length) {
    update(reinterpret_cast<const unsigned char*>(buf), length);
  }
  MD5& finalize() {
    if (!finalized_) {
      detail::check(qsmd5_ctx_final(ctx_, digest_), "qsmd5_ctx_final");
      finalized_ = true;
    }
    return *this;
  }
  // "" until finalize(), as MD5.cpp:318.
  std::string hexdigest() const { return finalized_ ? detail::hex(digest_) : std::string(); }
  friend std::ostream& operator<<(std::ostream& os, const MD5& m) { return os << m.hexdigest(); }

 private:
  qsmd5_ctx* ctx_ = nullptr;
  bool finalized_ = false;
  uint8_t digest_[16] = {0};
};

}  // namespace qsmd5

#ifndef QSMD5_NO_GLOBAL_MD5
// The reference declares md5() at global scope (MD5.h:95-96); so does this
// drop-in, unless QSMD5_NO_GLOBAL_MD5 is defined.
inline std::string md5(const std::string& str) { return qsmd5::md5(str); }
using MD5 = qsmd5::MD5;  // the reference's class, global as in MD5.h:51
template <class StreamPtr, qsmd5::detail::if_stream_ptr<StreamPtr> = 0>
inline std::string md5(const StreamPtr& stream) {
  return qsmd5::md5(stream);
}
#endif

#endif  // QSFS_AMD_QSFS_MD5_HPP_
