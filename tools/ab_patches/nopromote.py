"""A/B patch: tokenize.hip built without LLVM's private-array-to-LDS promotion (the marshal mode's promoted arrays
took 5 KiB of LDS per one-wave workgroup, halving K10's resident waves)."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "build.py")
    s = open(p).read()
    old = 'FILE_FLAGS = {"kernels.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]}'
    assert old in s
    open(p, "w").write(s.replace(old, 'FILE_FLAGS = {"kernels.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"], '
                                      '"tokenize.hip": ["-mllvm", "-disable-promote-alloca-to-lds"]}'))
