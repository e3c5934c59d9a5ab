#include <pybind11/pybind11.h>
namespace py = pybind11;
void bind_extra(py::module_& m) { (void)m; }
