"""Import the reference openpifpaf decoder from /root/reference (THIS CONTAINER ONLY).

TEST INFRASTRUCTURE.  Used by tests/golden/gen_golden.py to run the reference decoder and
record golden vectors.  Never imported by the product package, bench.py or the GPU tests
(/root/reference does not exist on the GPU box).

Two things stand between `import openpifpaf` and a working decoder here:
  * functional.pyx must be compiled: oracle/build_ref.sh builds it into oracle/_ref/;
    the module is registered as `openpifpaf.functional` before the package is imported.
  * torchvision is absent: openpifpaf/transforms/__init__.py:3 imports it at module level.
    No-op stubs are registered; the stubbed names are only used at import time or for NN
    construction, never by the decoder.
"""
import importlib.util
import os
import subprocess
import sys
import types

REF_ROOT = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))


def _stub_torchvision():
    if 'torchvision' in sys.modules:
        return
    tv = types.ModuleType('torchvision')
    tvt = types.ModuleType('torchvision.transforms')
    tvtf = types.ModuleType('torchvision.transforms.functional')
    tvm = types.ModuleType('torchvision.models')
    tvmr = types.ModuleType('torchvision.models.resnet')

    class _NoOp:
        def __init__(self, *args, **kwargs):
            pass

        def __call__(self, x, *args, **kwargs):
            return x

    for name in ('ToTensor', 'Normalize', 'ColorJitter', 'RandomGrayscale', 'Compose'):
        setattr(tvt, name, _NoOp)
    tvt.functional = tvtf
    tv.transforms = tvt
    tv.models = tvm
    tvm.resnet = tvmr
    sys.modules.update({
        'torchvision': tv,
        'torchvision.transforms': tvt,
        'torchvision.transforms.functional': tvtf,
        'torchvision.models': tvm,
        'torchvision.models.resnet': tvmr,
    })


def available():
    return os.path.isfile(os.path.join(REF_ROOT, 'openpifpaf', 'functional.pyx'))


def load():
    """Return the reference `openpifpaf` package (decoder importable)."""
    if 'openpifpaf' in sys.modules:
        return sys.modules['openpifpaf']
    if not available():
        raise RuntimeError('reference not present at ' + REF_ROOT)
    sys.dont_write_bytecode = True
    so_path = subprocess.check_output(
        ['bash', os.path.join(HERE, 'build_ref.sh')], text=True).strip().splitlines()[-1]
    spec = importlib.util.spec_from_file_location('openpifpaf.functional', so_path)
    functional = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(functional)
    sys.modules['openpifpaf.functional'] = functional
    _stub_torchvision()
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import openpifpaf  # noqa: E402  pylint: disable=import-outside-toplevel
    return openpifpaf
