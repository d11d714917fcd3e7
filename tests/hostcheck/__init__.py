"""TEST INFRASTRUCTURE ONLY: host build of the product's device physics headers."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(os.path.dirname(HERE), "_build", "libhostcheck.so")
_lib = None


def build_hostcheck():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", HERE])
        _lib = ctypes.CDLL(SO)
    return _lib
