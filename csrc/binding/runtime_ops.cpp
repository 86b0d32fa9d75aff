#include <torch/extension.h>
void register_runtime(pybind11::module& m) {}
