"""Build libpifpaf_amd.so (HIP, gfx950) in-tree: python -m openpifpaf_amd.build

Each csrc/*.hip compiles to an object with hipcc in parallel, then one shared library is
linked next to this file, so it travels with the repository snapshot to the GPU box.
-ffp-contract=off is part of the numerics contract (no FMA contraction).
"""
import concurrent.futures
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(REPO, 'build', 'hip')
LIB = os.path.join(HERE, 'libpifpaf_amd.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('PP_OFFLOAD_ARCH', 'gfx950')

CFLAGS = [
    '--offload-arch=' + ARCH, '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off',
    '-fno-fast-math', '-Wall', '-Wno-unused-function', '-I', os.path.join(REPO, 'include'),
]


# per-file flags: splat.hip's fold gains nothing from packed f32; without the SLP vectorizer
# the uniform CifHr runs 2-3 % faster (dense 5.41 -> 5.31 ms, sparse 4.36 -> 4.14-4.25 ms per
# 256 images, A/B on one box).  Hand-written packed folds measured slower too (dense uniform
# 5.48 -> 5.86-5.99 ms, profiles/r05p_fold_packed_ab.txt), although an isolated stream of
# v_pk_fma_f32 runs 1.6-1.9x the element rate of v_fma_f32 (tools/ubench/pk_rate.hip)
FILE_FLAGS = {'splat.hip': ['-fno-slp-vectorize']}


VARIANTS = {
    # the diagnostic build: per-section cycle stamps (tools/stamps_run.py, hr_stamps.py,
    # sort_stamps.py) and the PP_SPLIT_* overrides of tools/cfg2_split.py
    'stamps': ['-DPP_STAMPS'],
}
# Round 6 dropped the A/B variants whose changes lost (nofuse, noself, ahead, selfext, noocc,
# base, bitonic, parts8, w0plan, nopartial, hprio, radix7; DESIGN.md §4 has their numbers):
# the product library has no other build switch.  tools/src_variant.py builds a patched copy
# of csrc/ for new A/B runs.


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.hip'))


def source_digest():
    """sha256 (hex, 16 chars) of the library's sources (csrc/* and the C header): names a
    build, so that a committed profile can be matched with the library it measured."""
    import hashlib
    h = hashlib.sha256()
    paths = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                   if f.endswith(('.hip', '.hpp')))
    for p in paths + [os.path.join(REPO, 'include', 'pifpaf_amd.h')]:
        h.update(os.path.basename(p).encode() + b'\0')
        with open(p, 'rb') as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _deps_mtime():
    paths = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    paths.append(os.path.join(REPO, 'include', 'pifpaf_amd.h'))
    return max(os.path.getmtime(p) for p in paths)


def _compile(src, bdir=BUILD, extra=()):
    obj = os.path.join(bdir, os.path.basename(src)[:-4] + '.o')
    if os.path.exists(obj) and os.path.getmtime(obj) >= _deps_mtime():
        return obj
    cmd = [HIPCC] + CFLAGS + FILE_FLAGS.get(os.path.basename(src), []) + list(extra) + ['-c', src, '-o', obj]
    res = subprocess.run(cmd, capture_output=True, text=True, check=False)
    if res.returncode != 0:
        raise RuntimeError('hipcc failed for {}:\n{}\n{}'.format(src, ' '.join(cmd), res.stderr))
    return obj


def build(force=False, verbose=True, variant=''):
    """variant '' = the product library; 'stamps' = diagnostic build with in-kernel cycle
    stamps (-DPP_STAMPS), never loaded unless PP_LIB_VARIANT=stamps."""
    lib = LIB if not variant else LIB.replace('.so', '_{}.so'.format(variant))
    bdir = BUILD if not variant else BUILD + '_' + variant
    os.makedirs(bdir, exist_ok=True)
    if (not force and os.path.exists(lib) and os.path.getmtime(lib) >= _deps_mtime()):
        return lib
    # the diagnostic variant (never loaded by default): 'stamps' (in-kernel cycle stamps)
    extra = VARIANTS.get(variant, [])
    workers = min(8, len(sources()))
    with concurrent.futures.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(lambda src: _compile(src, bdir, extra), sources()))
    cmd = [HIPCC, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', lib] + objs
    res = subprocess.run(cmd, capture_output=True, text=True, check=False)
    if res.returncode != 0:
        raise RuntimeError('link failed:\n{}\n{}'.format(' '.join(cmd), res.stderr))
    if verbose:
        print('built', lib, file=sys.stderr)
    return lib


if __name__ == '__main__':
    build(force='--force' in sys.argv)
    if '--stamps' in sys.argv:
        build(force='--force' in sys.argv, variant='stamps')
    for v in sys.argv[1:]:
        if v.startswith('--variant='):
            build(force='--force' in sys.argv, variant=v.split('=', 1)[1])
