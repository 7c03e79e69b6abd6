"""Host-side timing of the bench step: where does the host spend time between launches?"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import _lib, codes, decoders  # noqa: E402

Hx, Hz = codes.load_code("LP118_0")
B = 1 << 20
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
sz = torch.randint(0, 2, (B, 240), dtype=torch.uint8, device=dev, generator=g)
sx = torch.randint(0, 2, (B, 240), dtype=torch.uint8, device=dev, generator=g)
mk = lambda: decoders.DecodeResult(torch.empty((B, 544), dtype=torch.uint8, device=dev),
                                   torch.empty(B, dtype=torch.int32, device=dev), None,
                                   torch.empty(B, dtype=torch.int32, device=dev))
oz, ox = mk(), mk()
for timing in (False, True):
    _lib.timing_enable(timing)
    for step in range(4):
        t0 = time.perf_counter()
        decoders.decode_batch(Hz, sz, 0.05 / 3, 50, algo="MS", out=oz)
        t1 = time.perf_counter()
        decoders.decode_batch(Hx, sx, 0.05 / 3, 50, algo="MS", out=ox)
        t2 = time.perf_counter()
        s = oz.iters.sum(dtype=torch.int64) + ox.iters.sum(dtype=torch.int64)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"timing={timing} step {step}: launchZ {1e3*(t1-t0):.2f} launchX {1e3*(t2-t1):.2f} "
              f"sum {1e3*(t3-t2):.2f} sync {1e3*(t4-t3):.2f} total {1e3*(t4-t0):.2f} ms", flush=True)
