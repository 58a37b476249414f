"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer: every
decode entry point over random fields at odd shapes (oracle/asan_main.c).  Host code only."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle')


@pytest.mark.skipif(shutil.which('gcc') is None, reason='needs gcc')
def test_oracle_under_asan_ubsan():
    subprocess.check_call(['make', '-s', '-C', ORACLE, 'asan'])
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0',
               UBSAN_OPTIONS='print_stacktrace=1')
    res = subprocess.run([os.path.join(ORACLE, 'asan_check')], env=env, capture_output=True,
                         text=True, timeout=600, check=False)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    assert 'asan ok' in res.stdout
