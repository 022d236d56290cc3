// qsfs-fuse_amd/tools/qsmd5sum.cpp -- per-part Content-MD5 of files, as qsfs
// would send them, computed in one GPU batch per invocation.
//
// This is the batch caller of SURVEY.md §8f row 1 in tool form:
//   1. slice each file into upload parts exactly like
//      QSTransferManager::PrepareUpload (QSTransferManager.cpp:475-550);
//   2. gather every part into pinned host memory -- the ResourceManager pool
//      (ResourceManager.cpp:53-77) made of qsmd5_alloc_pinned buffers;
//   3. hash all parts of all files in ONE qsmd5_hash_batch call instead of one
//      md5(buffer) per part (QSClient.cpp:370, 446).
//
// usage: qsmd5sum [-b MiB] [--parts] [--threshold MiB] [--min-part MiB] FILE...
//   default output: "<md5>  <file>" for files below the multipart threshold,
//   and one line per part for larger files (or for every file with --parts):
//   "<md5>  <file>#<part> <offset> <size>"
// Exit status: 0 ok, 1 usage or I/O error, 2 GPU error.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/qsmd5.h"

namespace {

struct FileParts {
  std::string path;
  uint64_t size = 0;
  std::vector<qsmd5_part> parts;
  uint8_t* data = nullptr;  // pinned
};

bool read_file(const char* path, FileParts& f, std::string& err) {
  FILE* fp = fopen(path, "rb");
  if (!fp) {
    err = std::string("cannot open ") + path;
    return false;
  }
  if (fseeko(fp, 0, SEEK_END) != 0) {
    fclose(fp);
    err = std::string("cannot seek ") + path;
    return false;
  }
  const off_t sz = ftello(fp);
  fseeko(fp, 0, SEEK_SET);
  f.path = path;
  f.size = (uint64_t)sz;
  void* p = nullptr;
  if (qsmd5_alloc_pinned(f.size ? f.size : 1, &p) != 0) {
    fclose(fp);
    err = std::string("pinned allocation failed: ") + qsmd5_last_error();
    return false;
  }
  f.data = static_cast<uint8_t*>(p);
  size_t got = f.size ? fread(f.data, 1, f.size, fp) : 0;
  fclose(fp);
  if (got != f.size) {
    err = std::string("short read ") + path;
    return false;
  }
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
    if (f.data) qsmd5_free_pinned(f.data);
  return rc;
}
