// tests/cpp/test_shim.cpp -- drop-in checks for qsfs-fuse_amd/host/qsfs_md5.hpp.
//
// Exercises the reference-shaped C++ interface on the GPU and prints one
// "name hexdigest" line per case; tests/test_gpu_shim.py compares every line
// with hashlib.  Also asserts the stream side effects of the reference
// md5(shared_ptr<iostream>) (MD5.cpp:343, 346: read position reset to 0) and
// the StreamBuf view contract (StreamBuf.cpp:32-48; StreamTest.cpp:131-150:
// a stream over a 3-byte buffer with lengthToRead=2 exposes "01").
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../qsfs-fuse_amd/host/qsfs_md5.hpp"

namespace {

// The qsfs StreamBuf contract: a view of the first `len` bytes of a shared
// vector<char> (StreamBuf.cpp:32-48), seekable (StreamBuf.cpp:56-91).
class ViewBuf : public std::streambuf {
 public:
  ViewBuf(std::shared_ptr<std::vector<char>> buf, size_t len) : buf_(std::move(buf)), len_(len) {
    char* b = buf_->data();
    setp(b, b + len_);
    setg(b, b, b + len_);
  }

 protected:
  pos_type seekoff(off_type off, std::ios_base::seekdir dir, std::ios_base::openmode which) override {
    if (dir == std::ios_base::beg) return seekpos(off, which);
    if (dir == std::ios_base::end) return seekpos(off_type(len_) - off, which);
    return seekpos((gptr() - eback()) + off, which);
  }
  pos_type seekpos(pos_type pos, std::ios_base::openmode) override {
    if (pos < 0 || pos > off_type(len_)) return pos_type(off_type(-1));
    char* b = buf_->data();
    setg(b, b + off_type(pos), b + len_);
    return pos;
  }

 private:
  std::shared_ptr<std::vector<char>> buf_;
  size_t len_;
};

class ViewStream : public std::iostream {
 public:
  ViewStream(std::shared_ptr<std::vector<char>> buf, size_t len) : std::iostream(nullptr), sb_(buf, len) {
    rdbuf(&sb_);
  }

 private:
  ViewBuf sb_;
};

std::vector<char> lcg(uint32_t seed, size_t n) {
  std::vector<char> v(n);
  uint32_t x = seed;
  for (size_t i = 0; i < n; ++i) {
    x = x * 1103515245u + 12345u;
    v[i] = static_cast<char>(x >> 16);
  }
  return v;
}

int failures = 0;
void expect(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    ++failures;
  }
}

}  // namespace

int main() {
  // The daemon's lifetime guard: init now, qsmd5_shutdown at the end of main.
  qsmd5::Runtime runtime;
  // 0. A shutdown in the middle re-initialises on the next call.
  {
    expect(md5(std::string("abc")) == "900150983cd24fb0d6963f7d28e17f72", "md5 before shutdown");
    expect(qsmd5_shutdown() == 0 && qsmd5_shutdown() == 0, "qsmd5_shutdown twice");
    expect(md5(std::string("abc")) == "900150983cd24fb0d6963f7d28e17f72", "md5 after shutdown");
  }
  // 1. md5(std::string) -- global, as the reference's free function.
  std::printf("str_empty %s\n", md5(std::string()).c_str());
  std::printf("str_abc %s\n", md5(std::string("abc")).c_str());
  std::printf("str_literal %s\n", md5("message digest").c_str());
  std::printf("content_md5_abc %s\n", qsmd5::content_md5_from_hex(md5(std::string("abc"))).c_str());

  // 2. md5(shared_ptr<iostream>) over a StreamBuf-style view (lengthToRead < size).
  for (size_t len : {size_t(0), size_t(2), size_t(55), size_t(64), size_t(10485760)}) {
    auto buf = std::make_shared<std::vector<char>>(lcg(12345, len + 100));
    std::shared_ptr<std::iostream> s = std::make_shared<ViewStream>(buf, len);
    s->seekg(7, std::ios_base::beg);  // position before the call must not matter
    std::string h = md5(s);
    std::printf("view_%zu %s\n", len, h.c_str());
    expect(s->tellg() == std::streampos(0), "read position reset to 0 after md5(stream)");
    expect(md5(s) == h, "md5(stream) is repeatable");
  }
  // StreamTest Read1: 3-byte buffer, lengthToRead = 2 -> hashes "01".
  {
    auto buf = std::make_shared<std::vector<char>>(std::vector<char>{'0', '1', '2'});
    std::shared_ptr<std::iostream> s = std::make_shared<ViewStream>(buf, 2);
    std::printf("streamtest_read1 %s\n", md5(s).c_str());
  }
  // 3. A stream whose get area is not the whole content (stringstream):
  //    falls back to reading through the streambuf.
  {
    std::shared_ptr<std::iostream> s = std::make_shared<std::stringstream>();
    std::string payload(100000, 'q');
    *s << payload;
    std::printf("stringstream_100000q %s\n", md5(s).c_str());
  }
  // 4. class MD5: update in pieces, finalize, hexdigest, operator<<.
  {
    std::vector<char> d = lcg(4242, 200000);
    qsmd5::MD5 m;
    expect(m.hexdigest().empty(), "hexdigest empty before finalize");
    size_t off = 0;
    for (unsigned cut : {63u, 1u, 64u, 65u, 199807u}) {
      m.update(d.data() + off, cut);
      off += cut;
    }
    m.finalize();
    std::ostringstream os;
    os << m;
    std::printf("class_pieces %s\n", os.str().c_str());
    qsmd5::MD5 one(std::string("abc"));
    std::printf("class_ctor_abc %s\n", one.hexdigest().c_str());
    // update after finalize: the reference keeps its digest (MD5.cpp:240-312)
    one.update("more", 4);
    one.finalize();
    expect(one.hexdigest() == "900150983cd24fb0d6963f7d28e17f72", "update after finalize is a no-op");
  }
  // 4b. The class is a value type, global as the reference's (MD5.h:51): a
  //     copy taken mid-stream hashes on by itself; copy-assignment, moves and
  //     operator<< by value (MD5.h:61) as any caller of the reference may use.
  {
    std::vector<char> d = lcg(31337, 5000);
    MD5 a;
    a.update(d.data(), 100);  // 100 B: one block hashed, 36 B pending in the tail
    MD5 b(a);
    b.update(d.data() + 100, 4900);
    a.update("x", 1);
    MD5 c;
    c = b;  // copy-assign a live context over a fresh one
    b.finalize();
    c.update("y", 1);
    std::printf("copy_b %s\n", b.hexdigest().c_str());
    std::printf("copy_a %s\n", a.finalize().hexdigest().c_str());
    std::printf("copy_c %s\n", c.finalize().hexdigest().c_str());
    MD5 moved(std::move(c));
    std::ostringstream os;
    auto by_value = [&os](MD5 m) { os << m; };  // the reference's operator<<(ostream&, MD5)
    by_value(moved);
    expect(os.str() == moved.hexdigest(), "a copied finalised MD5 prints its digest");
    MD5 fin(b);
    expect(fin.hexdigest() == b.hexdigest(), "a copy of a finalised MD5 keeps the digest");
  }
  // 5. Batch forms: md5_batch over ragged buffers, md5_file_parts over a
  //    25 MiB + 3 B "file" (PrepareUpload: 10, 10, 5 MiB + 3 B) and a 21 MiB one
  //    (10 MiB, then the 11 MiB remainder averaged into two 5.5 MiB parts).
  {
    std::vector<std::vector<char>> bufs;
    std::vector<qsmd5_chunk> chunks;
    for (size_t i = 0; i < 6; ++i) bufs.push_back(lcg(500 + (uint32_t)i, 1000 * i * i + 3 * i));
    for (auto& b : bufs) chunks.push_back(qsmd5_chunk{b.data(), b.size()});
    std::vector<std::string> hx = qsmd5::md5_batch(chunks);
    expect(hx.size() == bufs.size(), "md5_batch returns one digest per buffer");
    for (size_t i = 0; i < hx.size(); ++i) {
      std::printf("batch_%zu %s\n", i, hx[i].c_str());
      expect(hx[i] == qsmd5::md5_bytes(bufs[i].data(), bufs[i].size()), "md5_batch == md5_bytes");
    }
    for (uint64_t fsz : {uint64_t(25) * 1048576 + 3, uint64_t(21) * 1048576}) {
      std::vector<char> file = lcg(777, fsz);
      std::vector<qsmd5::PartMD5> parts = qsmd5::md5_file_parts(file.data(), file.size());
      uint64_t covered = 0;
      for (const auto& pm : parts) {
        std::printf("parts_%llu_%u %llu %llu %s\n", (unsigned long long)fsz, pm.part.part_number,
                    (unsigned long long)pm.part.offset, (unsigned long long)pm.part.size,
                    pm.md5.c_str());
        expect(pm.part.offset == covered, "parts are contiguous");
        expect(pm.md5 == qsmd5::md5_bytes(file.data() + pm.part.offset, pm.part.size),
               "md5_file_parts == md5 of the part bytes");
        covered += pm.part.size;
      }
      expect(covered == fsz, "parts cover the file");
    }
  }
  // 6. Errors are loud: NULL pointer with a non-zero length.
  {
    bool threw = false;
    try {
      qsmd5::md5_bytes(nullptr, 5);
    } catch (const qsmd5::Error& e) {
      threw = e.code() < 0;
    }
    expect(threw, "md5_bytes(NULL, 5) throws qsmd5::Error");
  }
  {
    bool threw = false;
    try {
      qsmd5::content_md5_from_hex("xyz");
    } catch (const qsmd5::Error&) {
      threw = true;
    }
    expect(threw, "content_md5_from_hex rejects non-hex text");
  }
  // 7. md5(stream) that fails (a malformed QSMD5_BACKEND makes every hashing
  //    call return -EINVAL) throws and still leaves the read position at 0.
  {
    const char* prev = getenv("QSMD5_BACKEND");
    const std::string saved = prev ? prev : "";
    setenv("QSMD5_BACKEND", "bogus", 1);
    auto buf = std::make_shared<std::vector<char>>(lcg(99, 4096));
    std::shared_ptr<std::iostream> s = std::make_shared<ViewStream>(buf, 4000);
    s->seekg(123, std::ios_base::beg);
    bool threw = false;
    try {
      md5(s);
    } catch (const qsmd5::Error& e) {
      threw = e.code() == -EINVAL;
    }
    if (prev) setenv("QSMD5_BACKEND", saved.c_str(), 1);
    else unsetenv("QSMD5_BACKEND");
    expect(threw, "md5(stream) throws qsmd5::Error(-EINVAL) on a hashing failure");
    expect(s->tellg() == std::streampos(0), "read position reset to 0 after a failed md5(stream)");
  }
  std::printf("failures %d\n", failures);
  return failures ? 1 : 0;
}
