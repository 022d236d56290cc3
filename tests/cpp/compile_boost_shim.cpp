// tests/cpp/compile_boost_shim.cpp -- compile-only check (tests/test_abi.py):
// the C++ drop-in accepts exactly the call qsfs makes, md5(buffer) with a
// boost::shared_ptr<std::iostream> (QSClient.cpp:370, 446), plus the string
// overload with a literal and class MD5 as the reference declares it.
#include <sstream>

#include "boost/shared_ptr.hpp"
#include "../../qsfs-fuse_amd/host/qsfs_md5.hpp"

std::string call_sites(boost::shared_ptr<std::iostream> buffer) {
  std::string a = md5(buffer);           // QSClient::UploadMultipart / UploadFile
  std::string b = md5(std::string("x"));  // md5(const std::string)
  std::string c = md5("literal");         // string literal -> std::string overload
  qsmd5::MD5 m;
  m.update("abc", 3u);
  return a + b + c + m.finalize().hexdigest();
}
