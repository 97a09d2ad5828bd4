"""Is a lone transform's pass bound by its workgroups running load / butterflies / store in
lockstep (one wave of 4-per-CU workgroups fills the chip exactly once)? Time S independent
dft calls issued on S streams at once against the same dft alone: if S concurrent
transforms take much less than S times as long, the pass kernels leave the chip idle
between phases, and a pipelined pass (or batching) is the lever, not the butterfly count.

usage (GPU): python tools/ntt_streams.py [log_n ...]     prints one line per (log_n, S)
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import dusk_plonk_amd as plk  # noqa: E402
from oracle_lib import random_fr  # noqa: E402  (sampler only)


def main():
    torch.cuda.set_device(0)
    ctx = plk.Context.default(0)
    for k in [int(a) for a in sys.argv[1:]] or [20, 23]:
        n = 1 << k
        fft = plk.Fft(k, ctx)
        S_MAX = 4
        xs = [torch.from_numpy(random_fr(n, 7 + i).view(np.int64)).cuda() for i in range(S_MAX)]
        ys = [torch.empty_like(x) for x in xs]
        scr = [torch.empty((2 * n, 4), dtype=torch.int64, device="cuda") for _ in range(S_MAX)]
        streams = [torch.cuda.Stream() for _ in range(S_MAX)]
        ref = None
        for S in (1, 2, 4):
            def burst():
                for i in range(S):
                    fft.ntt_dev(xs[i].data_ptr(), ys[i].data_ptr(), n, 1, False,
                                streams[i].cuda_stream, scr[i].data_ptr())
            for _ in range(3):
                burst()
            torch.cuda.synchronize()
            reps = 30
            t0 = time.perf_counter()
            for _ in range(reps):
                burst()
                torch.cuda.synchronize()  # bursts do not overlap each other
            dt = (time.perf_counter() - t0) / reps
            # the S outputs must agree with a lone transform of the same input
            if ref is None:
                ref = ys[0].clone()
            assert torch.equal(ys[0], ref)
            print(f"2^{k} S={S}: {dt * 1e3:.3f} ms per burst, {dt * 1e6 / S:.1f} us per transform",
                  flush=True)


if __name__ == "__main__":
    main()
