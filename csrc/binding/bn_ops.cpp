#include <torch/extension.h>
void register_bn_ops(pybind11::module& m) {}
