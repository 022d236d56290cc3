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
// --read: instead of mapping the files, let the library pull each part's
// bytes with pread(2) in column windows through its bounded pinned staging
// (qsmd5_hash_read, the pull-driven batch): the same one batch over every
// part, for files of any size, with at most --staging MiB staged at a time.
//
// usage: qsmd5sum [-b MiB] [--parts] [--threshold MiB] [--min-part MiB] [--read [--staging MiB]] FILE...
//   default output: "<md5>  <file>" for files below the multipart threshold,
//   and one line per part for larger files (or for every file with --parts):
//   "<md5>  <file>#<part> <offset> <size>"
// Exit status: 0 ok, 1 usage or I/O error, 2 GPU error.
#include <errno.h>
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
  int fd = -1;                    // --read: kept open for pread
};

// --read: chunk c of the batch is part `part` of file `file`
struct PartRef {
  const FileParts* file;
  uint64_t offset;
};

uint64_t pread_part(void* user, size_t chunk, uint64_t offset, uint64_t len, void* dst) {
  const PartRef& r = (*static_cast<const std::vector<PartRef>*>(user))[chunk];
  uint64_t done = 0;
  while (done < len) {
    const ssize_t got = pread(r.file->fd, static_cast<char*>(dst) + done, len - done,
                              (off_t)(r.offset + offset + done));
    if (got < 0 && errno == EINTR) continue;  // interrupted by a signal: not a short read
    if (got <= 0) break;  // EOF or an error: a short count fails the batch with -EIO
    done += (uint64_t)got;
  }
  return done;
}

bool open_file(const char* path, FileParts& f, std::string& err) {
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) {
    err = std::string("cannot open ") + path;
    return false;
  }
  struct stat st;
  if (fstat(f.fd, &st) != 0) {
    err = std::string("cannot stat ") + path;
    return false;
  }
  f.path = path;
  f.size = (uint64_t)st.st_size;
  (void)posix_fadvise(f.fd, 0, 0, POSIX_FADV_SEQUENTIAL);
  return true;
}

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
  uint64_t staging_mib = 0;  // --staging (0: the library's default)
  bool all_parts = false, pull = false;
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
    } else if (!strcmp(argv[i], "--read")) {
      pull = true;
    } else if (!strcmp(argv[i], "--staging") && i + 1 < argc) {
      staging_mib = strtoull(argv[++i], nullptr, 10);
    } else if (argv[i][0] == '-') {
      fprintf(stderr, "usage: %s [-b MiB] [--parts] [--threshold MiB] [--min-part MiB] "
              "[--read [--staging MiB]] FILE...\n", argv[0]);
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
    if (!(pull ? open_file(files[k], fs[k], err) : read_file(files[k], fs[k], err))) {
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
  if (rc == 0 && !chunks.empty() && pull) {
    std::vector<uint64_t> lens;
    std::vector<PartRef> refs;
    for (const FileParts& f : fs)
      for (const qsmd5_part& p : f.parts) {
        lens.push_back(p.size);
        refs.push_back({&f, p.offset});
      }
    // pread is thread-safe: let the library read a window's parts on several threads
    int e = qsmd5_hash_read(lens.data(), lens.size(), &pread_part, &refs, staging_mib * MiB,
                            reinterpret_cast<uint8_t(*)[16]>(dig.data()), QSMD5_FLAG_READ_PARALLEL);
    if (e != 0) {
      fprintf(stderr, "qsmd5sum: hashing failed: %s (%s)\n", qsmd5_strerror(e), qsmd5_last_error());
      rc = e == -EIO ? 1 : 2;
    }
  } else if (rc == 0 && !chunks.empty()) {
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
  for (FileParts& f : fs) {
    if (f.data) munmap(const_cast<uint8_t*>(f.data), f.size);
    if (f.fd >= 0) close(f.fd);
  }
  return rc;
}
