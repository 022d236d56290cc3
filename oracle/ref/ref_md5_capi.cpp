// oracle/ref/ref_md5_capi.cpp -- C entry points over the REFERENCE's own MD5.
//
// TEST INFRASTRUCTURE ONLY.  This translation unit is compiled together with
// the reference's src/base/MD5.cpp, read in place from /root/reference by
// oracle/build_ref.sh, into oracle/_ref/libref_md5.so (git-ignored; it
// travels to the GPU box as a built artefact, the reference source does not).
// It is used to (1) generate the golden fixtures under tests/golden/ and
// (2) serve as bench.py's cpu_baseline (kind "reference").
//
// Entry points wrap the two reference call forms:
//   md5(const std::string)                     MD5.h:95, MD5.cpp:335-339
//   md5(const boost::shared_ptr<iostream>&)    MD5.h:96, MD5.cpp:341-349
// The iostream form is fed through a get-area view over caller memory that
// exposes exactly `len` bytes, the same contract as qsfs's StreamBuf
// (src/data/StreamBuf.cpp:32-48: setg(begin, begin, begin + lengthToRead)).
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <iostream>
#include <streambuf>
#include <string>
#include <vector>

#include "MD5.h"  // reference header (include path set by build_ref.sh)

namespace {

// A read-only streambuf exposing [p, p+len) -- the StreamBuf contract.
class ViewBuf : public std::streambuf {
 public:
  ViewBuf(const char* p, size_t len) {
    char* b = const_cast<char*>(p);
    setg(b, b, b + len);
  }

 protected:
  pos_type seekoff(off_type off, std::ios_base::seekdir dir,
                   std::ios_base::openmode) override {
    char* target = nullptr;
    if (dir == std::ios_base::beg) target = eback() + off;
    else if (dir == std::ios_base::cur) target = gptr() + off;
    else target = egptr() - off;  // StreamBuf::seekoff(end) semantics
    if (target < eback() || target > egptr()) return pos_type(off_type(-1));
    setg(eback(), target, egptr());
    return pos_type(target - eback());
  }
  pos_type seekpos(pos_type pos, std::ios_base::openmode which) override {
    return seekoff(off_type(pos), std::ios_base::beg, which);
  }
};

void copy_hex(const std::string& h, char out[33]) {
  memset(out, 0, 33);
  memcpy(out, h.data(), h.size() < 32 ? h.size() : 32);
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) void ref_md5_string(const char* p, uint64_t len,
                                                           char out[33]) {
  copy_hex(md5(std::string(p, p + len)), out);
}

__attribute__((visibility("default"))) void ref_md5_iostream(const char* p, uint64_t len,
                                                             char out[33]) {
  ViewBuf vb(p, len);
  boost::shared_ptr<std::iostream> s(new std::iostream(&vb));
  copy_hex(md5(s), out);
}

// Streaming class API: MD5 m; m.update(...) in pieces; m.finalize().hexdigest()
// (MD5.h:55-61).  `cuts` are the piece lengths, summing to len.
__attribute__((visibility("default"))) void ref_md5_pieces(const char* p, const uint32_t* cuts,
                                                           size_t ncuts, char out[33]) {
  MD5 m;
  size_t off = 0;
  for (size_t i = 0; i < ncuts; ++i) {
    m.update(p + off, cuts[i]);
    off += cuts[i];
  }
  copy_hex(m.finalize().hexdigest(), out);
}

// Timed baseline: n chunks on nthreads threads, reference md5(std::string).
// `strings` are pre-built outside the timed region by ref_md5_prepare.
struct RefBatch {
  std::vector<std::string> strs;
};

__attribute__((visibility("default"))) void* ref_md5_prepare(const char* const* ptrs,
                                                             const uint64_t* lens, size_t n) {
  RefBatch* b = new RefBatch;
  b->strs.reserve(n);
  for (size_t i = 0; i < n; ++i) b->strs.emplace_back(ptrs[i], ptrs[i] + lens[i]);
  return b;
}

__attribute__((visibility("default"))) void ref_md5_release(void* h) {
  delete static_cast<RefBatch*>(h);
}

struct Job {
  RefBatch* b;
  char (*out)[33];
  std::atomic<size_t> next;
  int use_iostream;
};

static void* worker(void* arg) {
  Job* j = static_cast<Job*>(arg);
  for (;;) {
    size_t i = j->next.fetch_add(1);
    if (i >= j->b->strs.size()) break;
    const std::string& s = j->b->strs[i];
    if (j->use_iostream) {
      ref_md5_iostream(s.data(), s.size(), j->out[i]);
    } else {
      copy_hex(md5(s), j->out[i]);
    }
  }
  return nullptr;
}

__attribute__((visibility("default"))) int ref_md5_run(void* h, char (*out)[33], int nthreads,
                                                       int use_iostream) {
  Job j;
  j.b = static_cast<RefBatch*>(h);
  j.out = out;
  j.next = 0;
  j.use_iostream = use_iostream;
  if (nthreads < 1) nthreads = 1;
  std::vector<pthread_t> th;
  for (int t = 1; t < nthreads; ++t) {
    pthread_t x;
    if (pthread_create(&x, nullptr, worker, &j) == 0) th.push_back(x);
  }
  worker(&j);
  for (pthread_t x : th) pthread_join(x, nullptr);
  return 0;
}

}  // extern "C"
