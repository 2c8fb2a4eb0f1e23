"""A/B of patcher builds (scripts/build_variants.sh): every library named in AB_LIBS runs config 5's
ImagePatcher.convert_img_to_bag (7036 x 2800 synthetic mammogram, 224 px tiles, overlap 0.75,
empty_thresh 0.75, bf16 instances, shuffled) in its own process (MCGMIL_LIB), saves the bag and
reports its time; the parent checks the bags bitwise against the first library.
Usage: AB_LIBS=abvar/old.so,abvar/new.so python scripts/ab_patcher_libs.py"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out_dir):
    import torch
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
    from bench_cfg5 import H_IMG, OVERLAP, PS, THRESH, W_IMG, synthetic_mammogram
    from mcgmil.patcher import ImagePatcher
    dev = torch.device("cuda", 0)
    lib = os.path.basename(os.environ["MCGMIL_LIB"])
    img = synthetic_mammogram(dev, seed=5)
    p = ImagePatcher(patch_size=PS, overlap=OVERLAP, empty_thresh=THRESH)
    p.get_tiles(H_IMG, W_IMG)
    run = lambda: p.convert_img_to_bag(img, seed=0, out_dtype=torch.bfloat16)  # noqa: E731
    inst, ids, _ = run()
    torch.cuda.synchronize()
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    torch.save({"inst": inst.cpu(), "ids": torch.as_tensor(ids).cpu()}, os.path.join(out_dir, "bag.pt"))
    print(json.dumps({"lib": lib, "k": int(inst.shape[0]), "to_bag_ms": round(ms, 4),
                      "instance_GBps": round(inst.numel() * 2 / ms / 1e6, 1)}), flush=True)


def main():
    if os.environ.get("AB_CHILD"):
        return child(os.environ["AB_CHILD"])
    import torch
    libs = [q for q in os.environ["AB_LIBS"].split(",") if q]
    dirs = []
    for lib in libs:
        d = tempfile.mkdtemp(prefix="abpatch_")
        env = dict(os.environ, MCGMIL_LIB=os.path.abspath(lib), AB_CHILD=d)
        rc = subprocess.call([sys.executable, os.path.abspath(__file__)], env=env)
        if rc != 0:
            print(json.dumps({"lib": lib, "rc": rc}))
            return rc
        dirs.append(d)
    ref = torch.load(os.path.join(dirs[0], "bag.pt"), weights_only=True)
    ok = True
    for d, lib in zip(dirs[1:], libs[1:]):
        b = torch.load(os.path.join(d, "bag.pt"), weights_only=True)
        eq = torch.equal(b["ids"], ref["ids"]) and torch.equal(b["inst"].view(torch.int16), ref["inst"].view(torch.int16))
        ok &= eq
        if not eq:
            print(json.dumps({"lib": lib, "bitwise": False}))
    print(json.dumps({"bitwise_equal_all": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
