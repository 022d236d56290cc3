// qsfs-fuse_amd/tools/qsmd5sum.cpp -- per-part Content-MD5 of files, as qsfs
// would send them, computed in one GPU batch per invocation.
//
// This is the batch caller of SURVEY.md §8f row 1 in tool form:
//   1. slice each file into upload parts exactly like
//      QSTransferManager::PrepareUpload (QSTransferManager.cpp:475-550);
//   2. map each file (mmap, read-only): the batch's H2D copies read the page
//      cache directly, with no read() copy and no pinned buffer (pageable host
//      memory hashes as fast as pinned: DESIGN.md §5);
//   3. hash all parts of all files in ONE qsmd5_hash_batch call instead of one
//      md5(buffer) per part (QSClient.cpp:370, 446).
//
// usage: qsmd5sum [-b MiB] [--parts] [--threshold MiB] [--min-part MiB] FILE...
//   default output: "<md5>  <file>" for files below the multipart threshold,
//   and one line per part for larger files (or for every file with --parts):
//   "<md5>  <file>#<part> <offset> <size>"
// Exit status: 0 ok, 1 usage or I/O error, 2 GPU error.
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "../../include/qsmd5.h"

namespace {

struct FileParts {
  std::string path;
  uint64_t size = 0;
  std::vector<qsmd5_part> parts;
  const uint8_t* data = nullptr;  // the file, mapped read-only (nullptr when empty)
};

bool read_file(const char* path, FileParts& f, std::string& err) {
  const int fd = open(path, O_RDONLY);
  if (fd < 0) {
    err = std::string("cannot open ") + path;
    return false;
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    err = std::string("cannot stat ") + path;
    return false;
  }
  f.path = path;
  f.size = (uint64_t)st.st_size;
  if (f.size) {
    void* p = mmap(nullptr, f.size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (p == MAP_FAILED) {
      close(fd);
      err = std::string("cannot map ") + path;
      return false;
    }
    (void)madvise(p, f.size, MADV_SEQUENTIAL);
    (void)madvise(p, f.size, MADV_WILLNEED);  // start readahead of the whole file
    f.data = static_cast<const uint8_t*>(p);
  }
  close(fd);  // the mapping stays valid
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  uint64_t buf_mib = 10, threshold_mib = 20, min_part_mib = 4;  // configure/Default.cpp:159-177
  bool all_parts = false;
  std::vector<const char*> files;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "-b") && i + 1 < argc) {
      buf_mib = strtoull(argv[++i], nullptr, 10);
    } else if (!strcmp(argv[i], "--threshold") && i + 1 < argc) {
      threshold_mib = strtoull(argv[++i], nullptr, 10);
    } else if (!strcmp(argv[i], "--min-part") && i + 1 < argc) {
      min_part_mib = strtoull(argv[++i], nullptr, 10);
    } else if (!strcmp(argv[i], "--parts")) {
      all_parts = true;
    } else if (argv[i][0] == '-') {
      fprintf(stderr, "usage: %s [-b MiB] [--parts] [--threshold MiB] [--min-part MiB] FILE...\n",
              argv[0]);
      return 1;
    } else {
      files.push_back(argv[i]);
    }
  }
  if (files.empty() || buf_mib == 0) {
    fprintf(stderr, "usage: %s [-b MiB] [--parts] FILE...\n", argv[0]);
    return 1;
  }
  const uint64_t MiB = 1ull << 20;
  std::vector<FileParts> fs(files.size());
  std::vector<qsmd5_chunk> chunks;
  int rc = 0;
  for (size_t k = 0; k < files.size() && rc == 0; ++k) {
    std::string err;
    if (!read_file(files[k], fs[k], err)) {
      fprintf(stderr, "qsmd5sum: %s\n", err.c_str());
      rc = 1;
      break;
    }
    size_t n = 0;
    qsmd5_plan_parts(fs[k].size, buf_mib * MiB, min_part_mib * MiB, threshold_mib * MiB, 0,
                     nullptr, 0, &n);
    fs[k].parts.resize(n);
    if (qsmd5_plan_parts(fs[k].size, buf_mib * MiB, min_part_mib * MiB, threshold_mib * MiB, 0,
                         fs[k].parts.data(), n, &n) != 0) {
      fprintf(stderr, "qsmd5sum: planning failed: %s\n", qsmd5_last_error());
      rc = 1;
      break;
    }
    for (const qsmd5_part& p : fs[k].parts) chunks.push_back({fs[k].data + p.offset, p.size});
  }
  std::vector<uint8_t> dig(16 * chunks.size());
  if (rc == 0 && !chunks.empty()) {
    // the files were read into host memory: no per-part pointer query
    int e = qsmd5_hash_batch_ex(chunks.data(), chunks.size(),
                                reinterpret_cast<uint8_t(*)[16]>(dig.data()), QSMD5_FLAG_HOST);
    if (e != 0) {
      fprintf(stderr, "qsmd5sum: GPU hashing failed: %s (%s)\n", qsmd5_strerror(e),
              qsmd5_last_error());
      rc = 2;
    }
  }
  if (rc == 0) {
    size_t c = 0;
    for (const FileParts& f : fs) {
      const bool multi = all_parts || f.parts.size() > 1 || f.size >= threshold_mib * MiB;
      for (const qsmd5_part& p : f.parts) {
        char hex[33];
        qsmd5_hex(&dig[16 * c++], hex);
        if (multi)
          printf("%s  %s#%u %llu %llu\n", hex, f.path.c_str(), p.part_number,
                 (unsigned long long)p.offset, (unsigned long long)p.size);
        else
          printf("%s  %s\n", hex, f.path.c_str());
      }
    }
  }
  for (FileParts& f : fs)
    if (f.data) munmap(const_cast<uint8_t*>(f.data), f.size);
  return rc;
}
