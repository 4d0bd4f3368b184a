"""Builds the oracle's C++ restatement (checker / CPU baseline only) into
oracle/_build/liboracle.so with g++ (no HIP, no product code)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "liboracle.so")
SRCS = [os.path.join(HERE, "deepequal_ref.cpp"), os.path.join(HERE, "rollup_ref.cpp"), os.path.join(HERE, "csr_ref.cpp")]
DEPS = SRCS + [os.path.join(HERE, "xxh64_ref.h"), os.path.join(HERE, "timed_threads.h"), os.path.join(os.path.dirname(HERE), "include", "gpudiff_format.h"),
                os.path.join(os.path.dirname(HERE), "include", "gpudiff.h")]


def build() -> str:
    os.makedirs(OUT, exist_ok=True)
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(s) for s in DEPS):
        return LIB
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread"] + SRCS + ["-o", LIB]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)
    return LIB


if __name__ == "__main__":
    print(build())
