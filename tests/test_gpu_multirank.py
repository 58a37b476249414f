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
    assert 'multirank ok' in _run(world, [])[0]


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 3])
def test_sharded_api_matches_one_process(world):
    """CifCaf.decode_batch(group=) / Generator.batch(group=) over gloo ranks on cuda:0."""
    assert 'multirank ok' in _run(world, ['api'])[0]


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 3])
def test_cifdet_sharded_real_decode(world):
    """CifDet.decode_batch(group=) over gloo ranks on cuda:0 with the device decode (the
    CPU tests in test_distributed.py fake decode_records)."""
    assert 'multirank ok: det' in _run(world, ['det'])[0]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_cfg4_eight_ranks():
    """BASELINE.json configs[3] at full size: 2048 planted 80x80 images over 8 gloo ranks
    on cuda:0 (256 per rank, bench.py --workload cfg4's images), gathered on rank 0 with all
    8 digests verified, each shard byte-identical to its one-process decode and 4 images per
    shard checked against the oracle (tests/cfg4_worker.py).  8 ranks x (1.7 GB of fields +
    a 256-image workspace) fit the 288 GB of one MI355X."""
    import gc
    import torch
    gc.collect()  # this process's cached blocks from earlier tests go back to the device
    torch.cuda.empty_cache()
    outs = _run(8, [], worker='cfg4_worker.py', timeout=540, log_dir=os.path.join(
        os.path.dirname(HERE), 'gpurun_out', 'cfg4'))
    assert 'cfg4 ok: world 8, 2048 images' in outs[0]
    print(outs[0])


def _run(world, extra, worker='multirank_worker.py', timeout=100, log_dir=None):
    """Start `world` ranks of `worker` and wait for them; returns their outputs.  With
    `log_dir` each rank writes its output to a file there as it goes (a long run shows
    progress on disk), else into a pipe."""
    port = str(_free_port())
    procs, files = [], []
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=port, OMP_NUM_THREADS='2',
                   PYTHONUNBUFFERED='1')
        out = (open(os.path.join(log_dir, 'rank{}.log'.format(r)), 'w+') if log_dir else
               subprocess.PIPE)
        files.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, worker)] + extra,
                                      env=env, stdout=out, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p, f in zip(procs, files):
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        if f is not subprocess.PIPE:
            f.seek(0)
            out = f.read()
            f.close()
        outs.append(out)
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, 'rank {} failed:\n{}'.format(r, out[-3000:])
    return outs
