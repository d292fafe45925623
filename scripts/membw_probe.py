"""Write / read / copy bandwidth roofline of the box's HBM for the scan's sizes (torch fills,
copies and the fastest of several reductions for reads; median of 50 event-timed runs each)."""
import json
import torch


def timed(fn, reps=50):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for _ in range(5):
        fn()
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[reps // 2] * 1e3  # us


out = {}
for mb in (126, 512):
    n = mb * (1 << 20) // 4
    x = torch.empty(n, dtype=torch.int32, device="cuda")
    y = torch.empty_like(x)
    w = timed(lambda: x.fill_(7))
    c = timed(lambda: y.copy_(x))
    r = min(timed(lambda: x.sum(dtype=torch.int64)), timed(lambda: x.amax()),
            timed(lambda: x.view(torch.float32).sum()), timed(lambda: torch.count_nonzero(x)))
    out[f"{mb}MB"] = {"write_us": round(w, 1), "write_TBps": round(n * 4 / w / 1e6, 2),
                      "copy_us": round(c, 1), "copy_TBps_rw": round(2 * n * 4 / c / 1e6, 2),
                      "read_us": round(r, 1), "read_TBps": round(n * 4 / r / 1e6, 2)}
print(json.dumps(out))
