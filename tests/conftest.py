import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'oracle')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a HIP device (MI355X)')


@pytest.fixture(scope='session')
def lib_built():
    """Build libmamg.so and the oracle C library once (cross-compiles on CPU)."""
    import subprocess
    so = os.path.join(ROOT, 'metric-amg-examples_amd', 'libmamg.so')
    # the product library and the diagnosis build (same sources, -DMAMG_DIAG=1;
    # loaded only by child processes that test diagnosis switches)
    subprocess.check_call(['make', '-s', '-j8', '-C', os.path.join(ROOT, 'metric-amg-examples_amd', 'csrc'),
                           'all', 'diag'])
    subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'oracle')])
    assert os.path.exists(so)
    return so


def set_opt(name, value):
    """One of the library's internal layout switches for this process
    (mamg_set_option, include/mamg_test.h); reset after every test by
    _reset_options.  The product library reads no environment variables."""
    import metric_amg_examples_amd as M
    M._lib.set_option(name, value)
    _SET.add(name)


_SET = set()


@pytest.fixture(autouse=True)
def _reset_options():
    yield
    if _SET:
        import metric_amg_examples_amd as M
        for name in list(_SET):
            M._lib.set_option(name, None)
        _SET.clear()


DIAG_LIB = os.path.join(ROOT, 'metric-amg-examples_amd', 'libmamg_diag.so')


def diag_loaded():
    """True when this process loads the diagnosis build (MAMG_LIB)."""
    return os.path.realpath(os.environ.get('MAMG_LIB', '')) == os.path.realpath(DIAG_LIB)
