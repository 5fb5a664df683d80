import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tauv-vision_amd"), os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    # experiment builds only (tools/gpu_*.sh): run the suite against another build of the library
    # (make BUILD=build_x LIBDIR=lib_x EXTRA=...); the product reads no environment
    alt = os.environ.get("TV_TEST_LIB")
    if alt:
        from tauv_vision_amd import _lib
        _lib.set_library_path(os.path.abspath(alt))
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: multi-second CPU cases")
