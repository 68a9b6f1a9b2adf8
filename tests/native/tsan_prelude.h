// TEST-ONLY: force-included (-include) in every translation unit of the TSan builds: gcc
// 11's TSan does not intercept pthread_cond_clockwait, which libstdc++ uses for
// condition_variable::wait_for when this macro is set (see tsan_driver.cpp)
#pragma once
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
