"""TEST INFRASTRUCTURE -- builds the C part of the CPU oracle (oracle/philox_oracle.c).

Output goes to oracle/_build/liboracle.so (git-ignored, travels to the GPU box with the
snapshot). Called by __graft_entry__.build() and lazily by oracle.philox.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "philox_oracle.c")
OUT_DIR = os.path.join(HERE, "_build")
OUT = os.path.join(OUT_DIR, "liboracle.so")


def build(force: bool = False) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(SRC):
        return OUT
    tmp = OUT + ".tmp"
    subprocess.run(["gcc", "-O2", "-std=c99", "-Wall", "-Werror", "-shared", "-fPIC",
                    "-o", tmp, SRC, "-lm"], check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True))
