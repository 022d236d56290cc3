// qsfs-fuse_amd/csrc/qsmd5_vma.h -- which VMAs may be cached as host memory.
//
// Pure host logic, shared by the runtime's pointer classifier
// (qsmd5_rt.h Classifier) and the CPU test tests/cpp/test_vma.cpp.
//
// A pointer HIP does not know (pageable memory) is remembered by the VMA that
// holds it, so later chunks in that VMA skip the per-pointer query.  A VMA
// qualifies only if it is readable and anonymous ([heap], [stack], [anon:...]
// or no path) or a regular file outside /dev.  Device memory never lives in
// such a VMA: VRAM is an unreadable reservation or a mapping of a /dev file
// (/dev/dri/renderD*, /dev/kfd), dma-bufs are anon_inode mappings, and VMAs
// of different backing or permissions never merge.
#pragma once

#include <stdint.h>
#include <stdio.h>
#include <string.h>

namespace qsmd5 {

// Parses one /proc/<pid>/maps line ("lo-hi perms offset dev inode [path]").
// Returns true, with [*lo, *hi), if the VMA may be cached as host memory.
inline bool host_vma_from_maps_line(const char* line, uint64_t* lo, uint64_t* hi) {
  unsigned long long a = 0, b = 0;
  char perms[8] = {0};
  int path_at = 0;
  if (sscanf(line, "%llx-%llx %7s %*s %*s %*s %n", &a, &b, perms, &path_at) < 3) return false;
  if (path_at <= 0 || perms[0] != 'r' || b <= a) return false;
  const char* path = line + path_at;
  while (*path == ' ') ++path;
  const bool anon = *path == '\n' || *path == 0;
  const bool special = *path == '[' && (!strncmp(path, "[heap]", 6) || !strncmp(path, "[stack]", 7) ||
                                       !strncmp(path, "[anon:", 6));
  const bool file = *path == '/' && strncmp(path, "/dev/", 5) != 0;
  if (!(anon || special || file)) return false;
  *lo = a;
  *hi = b;
  return true;
}

}  // namespace qsmd5
