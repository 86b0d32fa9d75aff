#include <torch/extension.h>
void register_conv_ops(pybind11::module& m) {}
