"""Buffer lifetimes under poisoned memory.

A fresh child process with MAMG_POISON=1 set before it touches the GPU (every
double array a handle or the layout builder allocates starts as NaN bytes, so
a read of memory nothing wrote -- or a temporary freed under a kernel still
reading it and handed to the next allocation -- shows in the result) runs the
handle sequences that failed intermittently in round 3: several handles
built, applied, re-homed or not (MAMG_REHOME=0), K kernel variants, and the
half-symmetric / full SELL-64 pair with post fusion off.  Since round 4 the
setup's temporaries are freed in null-stream order (csrc/dmem.h), with no
device-wide drain.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = ('test_k_kernel_variants or test_half_symmetric_a0_bitwise or test_post_operator_k_equals_merged '
         'or test_multiple_handles_and_graph_cache or test_host_apply_after_queued_device_apply')


def _child(env, cases):
    cmd = [sys.executable, '-u', '-m', 'pytest', os.path.join(ROOT, 'tests', 'test_gpu.py'), '-q', '-x',
           '-p', 'no:cacheprovider', '--timeout', '200', '--timeout-method', 'thread', '-k', cases]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (p.stdout + p.stderr)[-3000:]
    assert p.returncode == 0, tail
    assert ' passed' in p.stdout and 'failed' not in p.stdout and 'skipped' not in p.stdout, tail


@pytest.mark.parametrize('mode', ['default', 'plain'])
def test_poisoned_handle_sequences_in_child(lib_built, mode):
    """default: the product's stream-ordered frees.  plain: MAMG_FREE_MODE=plain,
    hipMalloc / hipFree with no ordering of the library's own (the round-2
    code path): it must be as correct, since every setup kernel, copy and
    free is issued on the one (null) stream.  The child loads the diagnosis
    build (the same sources with the switches MAMG_FREE_MODE and
    MAMG_K_VARIANT compiled in; the product library reads neither)."""
    from conftest import DIAG_LIB
    env = dict(os.environ, MAMG_POISON='1', MAMG_LIB=DIAG_LIB)
    if mode == 'plain':
        env['MAMG_FREE_MODE'] = 'plain'
    _child(env, CASES)


def test_k_kernel_variants_in_child(lib_built):
    """The level-0 K kernel variants (1, 2, 4 lanes per row; MAMG_K_VARIANT)
    and their row-sorted slices, bitwise / against the oracle, in a child on
    the diagnosis build."""
    from conftest import DIAG_LIB
    _child(dict(os.environ, MAMG_LIB=DIAG_LIB), 'test_k_kernel_variants or test_k_row_sort_bitwise')
