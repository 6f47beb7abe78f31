"""ASan + UBSan run of the host C++ and the CPU oracle (SURVEY.md section 5;
VERDICT r04 #7).  tests/asan/host_asan.cpp drives setup.cpp, gen.cpp,
mms.cpp, convert.cpp and dist.cpp (every setup profile the host builds, the
BSR2 / SELL conversions, the row-partition plan for P = 2, 3, 4) and the
oracle's C cycle and PCG (oracle/vcycle_ref.c), all compiled with
-fsanitize=address,undefined -fno-sanitize-recover=all.  CPU only: the HIP
objects are not part of it (GPU sanitizers are not available on the box)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_under_asan_ubsan():
    d = os.path.join(ROOT, 'tests', 'asan')
    subprocess.check_call(['make', '-s', '-j8', '-C', d])
    env = dict(os.environ, OMP_NUM_THREADS='4', ASAN_OPTIONS='detect_leaks=1:abort_on_error=0',
               UBSAN_OPTIONS='print_stacktrace=1')
    p = subprocess.run([os.path.join(d, '_build', 'host_asan')], env=env, capture_output=True, text=True,
                       timeout=900)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert 'host_asan ok' in out, out[-4000:]
    assert 'AddressSanitizer' not in out and 'runtime error' not in out and 'LeakSanitizer' not in out, out[-4000:]
