// tests/cpp/integration_log_doctest.cpp -- compiles and runs INTEGRATION.md
// §2's log-sink binding as printed (tests/test_integration_doc.py cuts the
// block out: its two #include lines are dropped, the sink function goes to
// namespace scope, and the registration line runs in main).  The qsfs glog
// macros are test doubles here that record what they are given.
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/qsmd5.h"

static std::vector<std::string> g_lines;
#define DebugInfo(msg) g_lines.push_back(std::string("I ") + (msg))
#define DebugWarning(msg) g_lines.push_back(std::string("W ") + (msg))
#define DebugError(msg) g_lines.push_back(std::string("E ") + (msg))

#include LOG_SINK_FUNCTION

int main() {
#include LOG_SINK_REGISTRATION
  const char text[] = "abc";
  uint8_t d[16];
  if (qsmd5_hash_one(text, 3, d) != 0) return 1;
  for (const auto& l : g_lines) printf("%s\n", l.c_str());
  return 0;
}
