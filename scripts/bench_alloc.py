"""Where does the KV-cache allocation time go on a fresh box?  (p50 CR->ready breakdown)

Times torch.empty / zero_ of one 134 GB buffer (the default bench's KV pool), twice, then
the same bytes as 1 GB pieces, so the per-GB cost of hipMalloc (page mapping) vs the
zero fill is visible."""
import json
import time

import torch

GB = 1 << 30
dev = torch.device("cuda", 0)
torch.cuda.init()
torch.empty(1, device=dev)
torch.cuda.synchronize()
res = {}


def t(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, round(1e3 * (time.perf_counter() - t0), 1)


nbytes = 134 * GB
for rep in range(2):
    x, res[f"empty_134g_ms_{rep}"] = t(lambda: torch.empty(nbytes, dtype=torch.uint8, device=dev))
    _, res[f"zero_134g_ms_{rep}"] = t(lambda: x.zero_())
    _, res[f"zero_again_134g_ms_{rep}"] = t(lambda: x.zero_())
    del x
    _, res[f"free_empty_cache_ms_{rep}"] = t(torch.cuda.empty_cache)
pieces = []
t0 = time.perf_counter()
for i in range(134):
    pieces.append(torch.empty(GB, dtype=torch.uint8, device=dev))
    if i in (0, 7, 33):
        torch.cuda.synchronize()
        res[f"pieces_{i + 1}_ms"] = round(1e3 * (time.perf_counter() - t0), 1)
torch.cuda.synchronize()
res["pieces_134_ms"] = round(1e3 * (time.perf_counter() - t0), 1)
print(json.dumps(res), flush=True)
