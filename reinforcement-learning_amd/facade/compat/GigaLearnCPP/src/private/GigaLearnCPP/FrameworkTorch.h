// compat FrameworkTorch.h -- what src/ExampleMain.cpp takes from the reference's FrameworkTorch.h
// (GigaLearnCPP/src/private/GigaLearnCPP/FrameworkTorch.h) when it is compiled against the MI355X trainer facade:
// the GGL / RLGC surface (facade/GigaLearn.hpp) and the two torch names it calls, answered by the HIP runtime.
#pragma once
#include "GigaLearn.hpp"

namespace torch {
namespace cuda {
inline int device_count() {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}
inline bool is_available() { return device_count() > 0; }
}  // namespace cuda
}  // namespace torch

namespace c10 {
struct Error : std::exception {  // nothing here throws it; ExampleMain's handler only needs the type
    const char* what_without_backtrace() const noexcept { return what(); }
};
}  // namespace c10
