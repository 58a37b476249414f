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


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.hip'))


def _deps_mtime():
    paths = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    paths.append(os.path.join(REPO, 'include', 'pifpaf_amd.h'))
    return max(os.path.getmtime(p) for p in paths)


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src)[:-4] + '.o')
    if os.path.exists(obj) and os.path.getmtime(obj) >= _deps_mtime():
        return obj
    cmd = [HIPCC] + CFLAGS + ['-c', src, '-o', obj]
    res = subprocess.run(cmd, capture_output=True, text=True, check=False)
    if res.returncode != 0:
        raise RuntimeError('hipcc failed for {}:\n{}\n{}'.format(src, ' '.join(cmd), res.stderr))
    return obj


def build(force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    if (not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _deps_mtime()):
        return LIB
    workers = min(8, len(sources()))
    with concurrent.futures.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(_compile, sources()))
    cmd = [HIPCC, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', LIB] + objs
    res = subprocess.run(cmd, capture_output=True, text=True, check=False)
    if res.returncode != 0:
        raise RuntimeError('link failed:\n{}\n{}'.format(' '.join(cmd), res.stderr))
    if verbose:
        print('built', LIB, file=sys.stderr)
    return LIB


if __name__ == '__main__':
    build(force='--force' in sys.argv)
