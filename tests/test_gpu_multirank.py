"""Multi-rank decode on the GPU: N gloo ranks on cuda:0 decode
their shard() of one batch, gather compact records to rank 0, and rank 0 checks them
byte for byte against a one-process decode (tests/multirank_worker.py)."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 3])
def test_sharded_decode_gathers_one_process_result(world):
    _run(world, [])


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 3])
def test_sharded_api_matches_one_process(world):
    """CifCaf.decode_batch(group=) / Generator.batch(group=) over gloo ranks on cuda:0."""
    _run(world, ['api'])


def _run(world, extra):
    port = str(_free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, 'multirank_worker.py')] + extra,
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, 'rank {} failed:\n{}'.format(r, out[-3000:])
    assert 'multirank ok' in outs[0]
