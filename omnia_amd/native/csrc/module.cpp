// _omnia_native: host-side native runtime pieces (no GPU code).
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_aes_gcm(py::module_& m);
void register_json_grammar(py::module_& m);

PYBIND11_MODULE(_omnia_native, m) {
  m.doc() = "omnia_amd native host runtime (crypto, constrained-decoding grammar)";
  register_aes_gcm(m);
  register_json_grammar(m);
}
