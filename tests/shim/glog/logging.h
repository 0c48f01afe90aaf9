// Test-only glog stand-in for tests/test_dropin_cpu.py: the reference's test
// and CLI sources compile against the product's headers with this in place
// of <glog/logging.h> (LOG comes from frecsys/logging.h).
#pragma once
#include "frecsys/logging.h"
namespace google {
inline void InstallFailureSignalHandler() {}
inline void InitGoogleLogging(const char*) {}
}  // namespace google
