"""The multi-process half of the direct all-reduce (k_xar): exchange regions exported as IPC
handles, mapped by the other processes, and one self-test exchange over them -- what kb_comm_init sets up on a
multi-GPU node.  RCCL refuses several ranks on one device, so the mapping is exercised here with processes sharing
the one GPU (kb_xar_export / kb_xar_test, the hook that runs exactly the IPC and exchange code of kb_comm_init).

Bars: every rank's self-test exchange returns the exact rank-order sums (ok on all ranks); with a peer that does not
take part, the waiting rank's k_xar gives up after its wait bound (KB_XAR_TIMEOUT_MS, 2 s here; 10 s by default) and
reports failure (no hang)."""
import multiprocessing as mp
import os
import time

import pytest

pytestmark = pytest.mark.gpu

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, nranks, conn, participate):
    import sys
    sys.path.insert(0, _ROOT)
    from kalibr_amd import capi, synth
    try:
        s = capi.Solver(synth.make_config(4, n_frames=8, p_view=0.7))  # C = 106: the image path
        conn.send(s.xar_export())
        handles = conn.recv()
        if participate:
            t0 = time.time()
            ok = s.xar_test(nranks, rank, handles)
            conn.send((ok, time.time() - t0))
        else:
            conn.send((None, 0.0))
            conn.recv()  # stays alive (its region mapped by the peer) until released
        s.close()
    except Exception as e:  # reported to the parent instead of a silent child death
        conn.send(("error", repr(e)))


def _run(participates, timeout=180):
    ctx = mp.get_context("spawn")
    conns, procs = [], []
    n = len(participates)
    for r, part in enumerate(participates):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_rank, args=(r, n, b, part))
        p.start()
        conns.append(a)
        procs.append(p)
    try:
        hs = []
        for c in conns:
            assert c.poll(timeout), "a rank did not export its region"
            h = c.recv()
            assert isinstance(h, bytes), h
            hs.append(h)
        for c in conns:
            c.send(b"".join(hs))
        res = []
        for c in conns:
            assert c.poll(timeout), "a rank did not finish its exchange"
            res.append(c.recv())
        for c, part in zip(conns, participates):
            if not part:
                c.send("release")
        return res
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()


@pytest.mark.parametrize("nranks", [2, 3])
def test_ipc_exchange_between_processes(nranks):
    res = _run([True] * nranks)
    assert all(r[0] is True for r in res), res


def test_ipc_absent_peer_times_out(monkeypatch):
    monkeypatch.setenv("KB_XAR_TIMEOUT_MS", "2000")  # inherited by the spawned ranks
    res = _run([True, False])
    ok, sec = res[0]
    assert ok is False, res
    assert 1.5 < sec < 30.0, sec  # the 2 s wait bound, then a clean failure
