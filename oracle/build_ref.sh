#!/usr/bin/env bash
# Build the REFERENCE's own native primitive module (openpifpaf/functional.pyx) from the
# source where it lies under /root/reference, outputs only into oracle/_ref/ (git-ignored).
#
# TEST INFRASTRUCTURE ONLY.  The resulting extension is used in this container to
# (1) validate the C restatement in oracle/pp_oracle.c and (2) generate the golden
# fixtures under tests/golden/ (tests/golden/gen_golden.py).  It never ships with the
# product and the product never loads it.
#
# Recipe: Cython 3 translates functional.pyx (language_level 3) to C, gcc -O2 compiles it
# against the Python and NumPy headers.  The shipped functional.c (Cython 0.29) does not
# compile on Python 3.10 (functional.c:20727), so it is not used.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
SRC=/root/reference/openpifpaf/functional.pyx
OUT="$HERE/_ref"
if [ ! -f "$SRC" ]; then
  echo "reference not present ($SRC); skipping oracle/_ref build" >&2
  exit 0
fi
mkdir -p "$OUT"
PYINC=$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
NPINC=$(python3 -c 'import numpy; print(numpy.get_include())')
SUFFIX=$(python3 -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
if [ ! -f "$OUT/functional$SUFFIX" ] || [ "$SRC" -nt "$OUT/functional$SUFFIX" ]; then
  python3 -m cython -3 --module-name openpifpaf.functional "$SRC" -o "$OUT/functional.c"
  gcc -O2 -fPIC -shared -I"$PYINC" -I"$NPINC" "$OUT/functional.c" -o "$OUT/functional$SUFFIX" -lm
fi
echo "$OUT/functional$SUFFIX"
