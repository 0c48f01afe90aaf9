// Test-only fmt stand-in (tests/test_dropin_cpu.py): fmt::format comes from
// frecsys/logging.h.
#pragma once
#include "frecsys/logging.h"
