"""Host synthesis time of the bench circuit at 2^20: alone, and on a second thread while
the main thread proves (the bench's overlap), to locate contention."""
import concurrent.futures as cf
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from dusk_plonk_amd import plonk as plk  # noqa: E402
from dusk_plonk_amd.prover import Plonk, PlonkKey  # noqa: E402

k = 20
gates = (1 << k) - 14


def synth(seed):
    t = time.perf_counter()
    cs = Plonk()
    cs.synthetic_chain(gates, seed)
    return cs, time.perf_counter() - t


cs, _ = synth(1)
del cs
for r in range(3):
    cs, dt = synth(2 + r)
    del cs
    print(f"synth alone {dt * 1e3:.1f} ms", flush=True)
pool0 = cf.ThreadPoolExecutor(1)
for r in range(3):
    cs, dt = pool0.submit(synth, 30 + r).result()
    del cs
    print(f"worker thread, main waiting: synth {dt * 1e3:.1f} ms", flush=True)
for r in range(3):
    fut = pool0.submit(synth, 40 + r)
    time.sleep(0.08)
    cs, dt = fut.result()
    del cs
    print(f"worker thread, main sleeping: synth {dt * 1e3:.1f} ms", flush=True)
tau = np.array([5, 7, 11, 13], dtype=np.uint64)
pp = plk.PlonkParams.setup(k, tau)
cs, _ = synth(9)
prover, _ = PlonkKey.compile_composer(pp, b"probe", cs)
pool = cf.ThreadPoolExecutor(1)
for r in range(4):
    fut = pool.submit(synth, 20 + r)
    t = time.perf_counter()
    prover.prove_composer(cs, 100 + r)
    tp = time.perf_counter() - t
    cs2, dt = fut.result()
    print(f"overlapped: synth {dt * 1e3:.1f} ms, prove {tp * 1e3:.1f} ms", flush=True)
    del cs
    cs = cs2
for r in range(2):
    t = time.perf_counter()
    prover.prove_composer(cs, 200 + r)
    tp = time.perf_counter() - t
    print(f"prove alone {tp * 1e3:.1f} ms", flush=True)
