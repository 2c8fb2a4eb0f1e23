"""Host-side cost of one drop-in module call (infer.py:187-191's per-bag loop): cProfile over
repeated MultiHeadGatedAttentionMIL.mc_inference_features calls on one bag (N, T as bench.py's
single-bag line). Prints the top entries by own time and the mean wall time per call."""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))

import torch  # noqa: E402

from mcgmil import MultiHeadGatedAttentionMIL, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=False)
    sd = synthetic.head_state_dict(0, C=2, shared=False)
    own = m.state_dict()
    m.load_state_dict({k: torch.from_numpy(v).reshape(own[k].shape) for k, v in sd.items()}, strict=False)
    m.compute_dtype = torch.bfloat16
    m = m.to(dev).eval()
    H = torch.randn(2048, 512, device=dev).abs_().bfloat16()
    call = lambda i: m.mc_inference_features(H, T=100, seed=100 + i, return_stats=True)  # noqa: E731
    for i in range(20):
        call(i)
    torch.cuda.synchronize()
    n = 500
    torch.cuda._sleep(int(5e8))          # keep the GPU busy so the host never waits on it
    t0 = time.perf_counter()
    prof = cProfile.Profile()
    prof.enable()
    for i in range(n):
        call(i)
    prof.disable()
    host = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    print(f"host per call (under cProfile): {host * 1e6:.1f} us")
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
