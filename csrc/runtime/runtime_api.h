#pragma once
#include <pybind11/pybind11.h>

namespace fdt {
// Registers the native runtime classes (pinned H2D prefetcher, bucket planner, ...).
void register_runtime(pybind11::module_& m);
}  // namespace fdt
