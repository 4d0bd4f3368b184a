"""A/B builds on one GPU box: each variant is a real source tree (so its build ID is its own sources' hash),
built in-tree here and shipped with the snapshot; tools/ab_tree.py run times them one process at a time, interleaved
over rounds, on the same box.

    python tools/ab_tree.py make NAME [--rev REV] [--patch FILE]   # ab/NAME from git REV (default: the working tree)
    python tools/ab_tree.py run NAME1,NAME2,... --config config2 [--rounds 3] [--pairs N] [--script bench.py] [-- args]

--patch FILE: a Python file with `def patch(root)` that edits the tree's sources before the build.  `.` as a NAME in
run is the repo itself.  ab/ is git-ignored; delete it when done (it is shipped to the GPU box while it exists).
"""
import argparse
import importlib.util
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB = os.path.join(ROOT, "ab")
PARTS = ["kcp_amd", "include", "tools/k2_time.py", "bench.py", "bench_upsert.py", "bench_rollup.py", "bench_negotiate.py",
         "bench_replay.py"]


def make(name, rev, patch):
    dst = os.path.join(AB, name)
    if os.path.exists(dst):
        shutil.rmtree(dst)
    os.makedirs(dst)
    if rev:
        tracked = subprocess.run(["git", "ls-tree", "--name-only", rev] + PARTS, cwd=ROOT, capture_output=True,
                                 text=True, check=True).stdout.split()
        tar = subprocess.run(["git", "archive", rev] + tracked, cwd=ROOT, capture_output=True, check=True).stdout
        subprocess.run(["tar", "-x", "-C", dst], input=tar, check=True)
        os.makedirs(os.path.join(dst, "tools"), exist_ok=True)
        shutil.copy(os.path.join(ROOT, "tools", "k2_time.py"), os.path.join(dst, "tools", "k2_time.py"))
    else:
        for p in PARTS:
            s, d = os.path.join(ROOT, p), os.path.join(dst, p)
            if os.path.isdir(s):
                shutil.copytree(s, d, ignore=shutil.ignore_patterns("_build", "__pycache__", "*.so", "*.stamp"))
            else:
                os.makedirs(os.path.dirname(d), exist_ok=True)
                shutil.copy(s, d)
    if patch:
        spec = importlib.util.spec_from_file_location("_ab_patch", patch)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.patch(dst)
    r = subprocess.run([sys.executable, os.path.join(dst, "kcp_amd", "build.py")], capture_output=True, text=True)
    if r.returncode:
        sys.exit("build of %s failed:\n%s%s" % (name, r.stdout[-3000:], r.stderr[-3000:]))
    shutil.rmtree(os.path.join(dst, "kcp_amd", "_build"), ignore_errors=True)  # objects are not shipped
    print("ab/%s built" % name)


def run(names, config, rounds, pairs, extra, timeout, script):
    # the tree's own package first (its script's directory), the main repo after it for oracle/ and tests/
    env = dict(os.environ, KCP_AB_MAIN=ROOT, PYTHONPATH=ROOT)
    for r in range(rounds):
        for nm in names:
            tree = ROOT if nm == "." else os.path.join(AB, nm)
            cmd = [sys.executable, os.path.join(tree, script), "--config", config] + (
                ["--pairs", str(pairs)] if pairs else []) + extra
            t0 = time.time()
            p = subprocess.run(cmd, cwd=tree, env=env, capture_output=True, text=True, timeout=timeout)
            if p.returncode:
                print(json.dumps({"variant": nm, "round": r, "rc": p.returncode, "err": p.stderr[-1500:]}), flush=True)
                sys.exit(1)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            d.update(variant=nm, round=r, wall_s=round(time.time() - t0, 1))
            print(json.dumps(d), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["make", "run"])
    ap.add_argument("names")
    ap.add_argument("--rev", default="")
    ap.add_argument("--patch", default="")
    ap.add_argument("--config", default="config2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=0)
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("--script", default="tools/k2_time.py", help="e.g. bench.py (any script printing a JSON line)")
    args, extra = ap.parse_known_args()
    extra = [a for a in extra if a != "--"]
    if args.cmd == "make":
        make(args.names, args.rev, args.patch)
    else:
        run(args.names.split(","), args.config, args.rounds, args.pairs, extra, args.timeout, args.script)


if __name__ == "__main__":
    main()
