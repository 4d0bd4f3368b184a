"""kcp_amd/csrc/pool.h (the context's host worker pool): an exception thrown on a worker thread (e.g.
std::bad_alloc in a growing vector) is carried back to run()'s caller -- whose catch turns it into
GPUDIFF_E_NOMEM -- instead of leaving the thread and calling std::terminate."""
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r'''
#include "pool.h"
#include <cstdio>
#include <new>
#include <stdexcept>
int main() {
    gd::WorkerPool p(8);
    int caught = 0;
    for (int rep = 0; rep < 50; rep++) {
        for (uint32_t bad = 0; bad < 8; bad++) {
            try {
                p.run(8, [&](uint32_t t) { if (t == bad) throw std::bad_alloc(); });
            } catch (const std::bad_alloc&) { caught++; }
        }
        // the pool still works afterwards
        std::atomic<int> n{0};
        p.run(8, [&](uint32_t) { n++; });
        if (n != 8) { std::printf("bad count %d\n", (int)n); return 1; }
    }
    std::printf("%d\n", caught);
    return caught == 400 ? 0 : 2;
}
'''


def test_worker_exception_reaches_caller():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "t.cpp")
        exe = os.path.join(d, "t")
        with open(src, "w") as f:
            f.write(SRC)
        subprocess.run(["g++", "-O1", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "kcp_amd", "csrc"),
                        "-include", "atomic", src, "-o", exe], check=True)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
        assert r.stdout.strip() == "400"
