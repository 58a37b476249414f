"""A/B builds that change a constant of the library source without touching csrc/: copies
csrc/ to build_src_<name>/, applies literal replacements, and links
openpifpaf_amd/libpifpaf_amd_<name>.so (PP_LIB_VARIANT=<name> loads it).
Usage: python tools/src_variant.py <name> <file> '<old>' '<new>' [<file> '<old>' '<new>' ...]
('<old>' must occur once; '*<old>' replaces every occurrence)"""
import os
import shutil
import subprocess
import sys
import concurrent.futures

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import build as B  # noqa: E402


def main():
    name, rest = sys.argv[1], sys.argv[2:]
    src_dir = os.path.join(B.REPO, 'build_src_' + name)
    shutil.rmtree(src_dir, ignore_errors=True)
    shutil.copytree(B.CSRC, src_dir)
    for i in range(0, len(rest), 3):
        p = os.path.join(src_dir, rest[i])
        s = open(p).read()
        old = rest[i + 1]
        if old.startswith('*'):  # '*<text>': every occurrence (at least one)
            old = old[1:]
            assert s.count(old) >= 1, (rest[i], old)
        else:
            assert s.count(old) == 1, (rest[i], old, s.count(old))
        open(p, 'w').write(s.replace(old, rest[i + 2]))
    bdir = src_dir + '/obj'
    os.makedirs(bdir)
    srcs = sorted(os.path.join(src_dir, f) for f in os.listdir(src_dir) if f.endswith('.hip'))

    def comp(src):
        obj = os.path.join(bdir, os.path.basename(src)[:-4] + '.o')
        cmd = [B.HIPCC] + B.CFLAGS + B.FILE_FLAGS.get(os.path.basename(src), []) + ['-c', src, '-o', obj]
        subprocess.run(cmd, check=True, capture_output=True)
        return obj
    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(comp, srcs))
    lib = B.LIB.replace('.so', '_{}.so'.format(name))
    subprocess.run([B.HIPCC, '--offload-arch=' + B.ARCH, '-shared', '-fPIC', '-o', lib] + objs, check=True)
    print('built', lib)


if __name__ == '__main__':
    main()
