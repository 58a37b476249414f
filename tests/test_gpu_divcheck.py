"""div_refined (the CifHr fold's hoisted-reciprocal division) equals the compiler's IEEE
f32 division bit for bit on its domain: builds and runs tests/hip/div_check.hip."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_div_refined_bit_exact(tmp_path):
    exe = str(tmp_path / 'div_check')
    subprocess.check_call(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17',
                           '-ffp-contract=off', '-I', os.path.join(HERE, '..', 'include'),
                           os.path.join(HERE, 'hip', 'div_check.hip'), '-o', exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300, check=False)
    assert out.returncode == 0, out.stdout + out.stderr
    assert 'mismatches 0' in out.stdout
