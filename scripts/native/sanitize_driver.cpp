// Sanitizer driver for the host-native C++: the pybind11 module
// sources are compiled INTO this executable with -fsanitize=address,undefined,
// registered as a builtin module, and exercised by the repo's own Python tests
// (AES-GCM NIST vectors, guided-decoding grammar) inside an embedded
// interpreter -- so every native call those tests make runs instrumented.
#include <Python.h>

#include <cstdio>
#include <string>

extern "C" PyObject* PyInit__omnia_native();

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <repo_root> <pytest args...>\n", argv[0]);
    return 2;
  }
  PyImport_AppendInittab("_omnia_native", &PyInit__omnia_native);
  Py_Initialize();
  std::string root = argv[1];
  std::string args = "[";
  for (int i = 2; i < argc; ++i) args += "r'" + std::string(argv[i]) + "',";
  args += "]";
  std::string code =
      "import sys\n"
      "sys.path.insert(0, r'" + root + "')\n"
      "import _omnia_native\n"
      "sys.modules['omnia_amd.native._omnia_native'] = _omnia_native\n"
      "print('native module:', getattr(_omnia_native, '__file__', '<builtin, sanitized>'))\n"
      "import pytest\n"
      "rc = pytest.main(" + args + ")\n"
      "sys.exit(int(rc))\n";
  int rc = PyRun_SimpleString(code.c_str());
  // PyRun_SimpleString returns -1 on an unhandled exception, including SystemExit
  // which it already reported; fetch the exit code through sys
  if (Py_FinalizeEx() < 0) return 120;
  return rc;
}
