"""openpifpaf_amd — MI355X (gfx950) drop-in for openpifpaf's CIF/CAF decoder hot path.

  openpifpaf_amd.functional   <- openpifpaf.functional (functional.pyx primitives)
  openpifpaf_amd.decoder      <- openpifpaf.decoder {CifHr, CifSeeds, CafScored, CifCaf, ...}
  openpifpaf_amd.Annotation   <- openpifpaf.Annotation

Compute runs in hand-written HIP kernels (libpifpaf_amd.so, C ABI in include/pifpaf_amd.h);
torch provides device memory and streams.
"""
__version__ = '0.1.0'
REFERENCE_VERSION = '0.11.6'

from .annotation import Annotation  # noqa: E402
