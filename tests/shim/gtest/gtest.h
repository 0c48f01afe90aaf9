// Test-only googletest stand-in (tests/test_dropin_cpu.py): enough of the
// TEST / TEST_F / EXPECT_* surface for the reference's tests/*_test.cc to
// compile (-fsyntax-only) against the product's headers.
#pragma once
#include <cmath>
#include <string>
namespace testing {
class Test {
 public:
  virtual ~Test() = default;
 protected:
  virtual void SetUp() {}
  virtual void TearDown() {}
  virtual void TestBody() = 0;
};
struct AssertSink {
  template <typename T>
  AssertSink& operator<<(const T&) { return *this; }
};
}  // namespace testing
#define GTEST_SHIM_CLASS_(suite, name) suite##_##name##_Test
#define TEST_F(suite, name)                                        \
  class GTEST_SHIM_CLASS_(suite, name) : public suite {            \
   protected:                                                      \
    void TestBody() override;                                      \
  };                                                               \
  void GTEST_SHIM_CLASS_(suite, name)::TestBody()
#define TEST(suite, name)                                                   \
  class GTEST_SHIM_CLASS_(suite, name) : public ::testing::Test {           \
   protected:                                                               \
    void TestBody() override;                                               \
  };                                                                        \
  void GTEST_SHIM_CLASS_(suite, name)::TestBody()
#define GTEST_SHIM_CHECK_(cond) if (!(cond)) ::testing::AssertSink()
#define EXPECT_TRUE(a) GTEST_SHIM_CHECK_(a)
#define EXPECT_FALSE(a) GTEST_SHIM_CHECK_(!(a))
#define EXPECT_EQ(a, b) GTEST_SHIM_CHECK_((a) == (b))
#define EXPECT_NE(a, b) GTEST_SHIM_CHECK_((a) != (b))
#define EXPECT_LE(a, b) GTEST_SHIM_CHECK_((a) <= (b))
#define EXPECT_LT(a, b) GTEST_SHIM_CHECK_((a) < (b))
#define EXPECT_GE(a, b) GTEST_SHIM_CHECK_((a) >= (b))
#define EXPECT_GT(a, b) GTEST_SHIM_CHECK_((a) > (b))
#define EXPECT_NEAR(a, b, e) GTEST_SHIM_CHECK_(std::fabs((a) - (b)) <= (e))
#define ASSERT_TRUE(a) EXPECT_TRUE(a)
#define ASSERT_EQ(a, b) EXPECT_EQ(a, b)
#define ASSERT_LE(a, b) EXPECT_LE(a, b)
#define ASSERT_NEAR(a, b, e) EXPECT_NEAR(a, b, e)
