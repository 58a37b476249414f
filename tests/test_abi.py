"""The C-ABI library loads and exports every symbol include/pifpaf_amd.h declares, and the
record layouts the Python side assumes match the C structs.  No GPU needed."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from openpifpaf_amd import _abi, _lib

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
HEADER = os.path.join(REPO, 'include', 'pifpaf_amd.h')


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(pp_[a-z0-9_]+)\s*\(', text)))


@pytest.fixture(scope='module')
def lib():
    from openpifpaf_amd import build
    build.build(verbose=False)
    return _lib.load()


def test_every_declared_symbol_exported(lib):
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes table covers every declaration
    assert set(names) == set(_lib.EXPORTED), set(names) ^ set(_lib.EXPORTED)


def test_version_and_defaults(lib):
    assert lib.pp_version() == _abi.PP_ABI_VERSION
    cfg = _abi.PPConfig()
    lib.pp_default_config(ctypes.byref(cfg))
    ref = _abi.make_config()
    for name, typ in _abi.PPConfig._fields_:
        if issubclass(typ, ctypes._Pointer):  # confidence_scales: NULL in both
            assert not getattr(cfg, name) and not getattr(ref, name), name
            continue
        assert getattr(cfg, name) == pytest.approx(getattr(ref, name)), name


def test_pitch_and_workspace_sizes(lib):
    assert lib.pp_cifhr_pitch(633) == 640
    assert lib.pp_cifhr_pitch(1273) == 1280
    assert lib.pp_cifhr_pitch(641) == 672
    cfg = _abi.make_config()
    size = lib.pp_decode_workspace_size(256, 17, 19, 80, 80, ctypes.byref(cfg), 800)
    zoff = lib.pp_decode_workspace_zero_offset(256, 17, 19, 80, 80, ctypes.byref(cfg), 800)
    assert 0 < zoff < size
    assert lib.pp_decode_workspace_size(0, 17, 19, 80, 80, ctypes.byref(cfg), 800) >= 0
    assert lib.pp_decode_workspace_size(1, 0, 19, 80, 80, ctypes.byref(cfg), 800) == 0


def test_argument_errors_without_gpu(lib):
    cfg = _abi.make_config()
    rc = lib.pp_cifhr(None, 1, 17, 8, 8, ctypes.byref(cfg), None, None, 0, None)
    assert rc == -1
    assert b'NULL' in lib.pp_last_error()
    dummy = ctypes.c_void_p(16)
    rc = lib.pp_cifhr(dummy, 1, 0, 8, 8, ctypes.byref(cfg), dummy, dummy, 1 << 20, None)
    assert rc == -2


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / 'layout.c'
    src.write_text('''
#include <stdio.h>
#include <stddef.h>
#include "pifpaf_amd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(pp_ann), offsetof(pp_ann, score),
         offsetof(pp_ann, decoding_pairs), offsetof(pp_ann, decoding_xyv),
         offsetof(pp_ann, frontier_pairs), sizeof(pp_seed), sizeof(pp_config),
         offsetof(pp_ann, n_frontier), offsetof(pp_config, exp_mode));
  return 0;
}
''')
    exe = tmp_path / 'layout'
    subprocess.check_call(['gcc', '-I', os.path.dirname(HEADER), str(src), '-o', str(exe)])
    vals = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    d = _abi.ANN_DTYPE
    assert vals == [d.itemsize, d.fields['score'][1], d.fields['decoding_pairs'][1],
                    d.fields['decoding_xyv'][1], d.fields['frontier_pairs'][1],
                    _abi.SEED_DTYPE.itemsize, ctypes.sizeof(_abi.PPConfig),
                    d.fields['n_frontier'][1], _abi.PPConfig.exp_mode.offset]


def test_no_oracle_in_product():
    """The product package never imports or links the oracle (test infrastructure)."""
    pkg = os.path.join(REPO, 'openpifpaf_amd')
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(('.py', '.hip', '.hpp', '.cpp')):
                text = open(os.path.join(root, f)).read()
                assert 'oracle' not in text.replace('Oracle', '').lower() or f == 'build.py', f


def test_det_struct_layout_matches_header(tmp_path):
    src = tmp_path / 'det_layout.c'
    src.write_text('''
#include <stdio.h>
#include <stddef.h>
#include "pifpaf_amd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(pp_det), offsetof(pp_det, score),
         offsetof(pp_det, bbox), offsetof(pp_det, image), sizeof(pp_det_nms),
         offsetof(pp_det_nms, apply));
  return 0;
}
''')
    exe = tmp_path / 'det_layout'
    subprocess.check_call(['gcc', '-I', os.path.dirname(HEADER), str(src), '-o', str(exe)])
    vals = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    d = _abi.DET_DTYPE
    assert vals == [d.itemsize, d.fields['score'][1], d.fields['bbox'][1], d.fields['image'][1],
                    ctypes.sizeof(_abi.DetNms), _abi.DetNms.apply.offset]


def test_scale_struct_and_multi_workspace():
    """pp_scale layout and the host-only multi-scale sizing entry points (no GPU needed)."""
    import ctypes
    from openpifpaf_amd._abi import ROLE_CAF, ROLE_CIF, Scale, make_config, scale_list
    from openpifpaf_amd._lib import load
    assert ctypes.sizeof(Scale) == 48
    lib = load()
    cfg = make_config()
    arr = scale_list([(0, 41, 41), (0, 21, 21)], [(0, 41, 41), (0, 21, 21)], [8, 16], [8, 16],
                     [0.0, 12.0], [0.0, 36.0], [160.0, None])
    assert [s.role for s in arr] == [ROLE_CIF, ROLE_CIF, ROLE_CAF, ROLE_CAF]
    size = lib.pp_decode_multi_workspace_size(arr, 4, 0, 2, 17, 19, ctypes.byref(cfg), 128)
    zero = lib.pp_decode_multi_workspace_zero_offset(arr, 4, 0, 2, 17, 19, ctypes.byref(cfg), 128)
    assert 0 < zero < size
    # one CIF + one CAF head of the single-scale shape sizes like pp_decode_workspace_size
    one = scale_list([(0, 41, 41)], [(0, 41, 41)], [8], [8])
    assert (lib.pp_decode_multi_workspace_size(one, 2, 0, 2, 17, 19, ctypes.byref(cfg), 128)
            == lib.pp_decode_workspace_size(2, 17, 19, 41, 41, ctypes.byref(cfg), 128))
    # ... and puts its working records at the same place (pp_decode_initial into a
    # single-scale engine workspace; CifCaf reads NMS-dropped initial annotations there)
    work = lib.pp_decode_work_offset(2, 17, 19, 41, 41, ctypes.byref(cfg), 128)
    assert 0 < work < lib.pp_decode_workspace_size(2, 17, 19, 41, 41, ctypes.byref(cfg), 128)
    assert work == lib.pp_decode_multi_work_offset(one, 2, 0, 2, 17, 19, ctypes.byref(cfg), 128)
    # pairs need an even CIF head count; no CAF head is rejected
    odd = scale_list([(0, 41, 41)] * 3, [(0, 41, 41)], [8] * 3, [8])
    assert lib.pp_decode_multi_workspace_size(odd, 4, 1, 1, 17, 19, ctypes.byref(cfg), 128) == 0
    cif_only = scale_list([(0, 41, 41)], [], [8], [])
    assert lib.pp_decode_multi_workspace_size(cif_only, 1, 0, 1, 17, 19, ctypes.byref(cfg), 128) == 0
    assert lib.pp_cifhr_multi_workspace_size(cif_only, 1, 0, 1, 17) > 0


def test_packed_record_size_matches_python_layout():
    """pp_packed_record_size (a host function) agrees with _abi.packed_dtype for every flag
    set, COCO and dense skeletons; compact records are at least 2x smaller than pp_ann."""
    from openpifpaf_amd._abi import ANN_DTYPE, packed_dtype
    lib = _lib.load()
    for k, c in ((17, 19), (17, 44), (24, 64), (1, 1), (5, 3)):
        for flags in (0, 1, 2, 3):
            assert lib.pp_packed_record_size(k, c, flags) == packed_dtype(k, c, flags).itemsize
            assert packed_dtype(k, c, flags).itemsize % 16 == 0
    assert lib.pp_packed_record_size(0, 19, 3) == 0 and lib.pp_packed_record_size(17, 65, 3) == 0
    assert 2 * packed_dtype(17, 19, 3).itemsize < ANN_DTYPE.itemsize
