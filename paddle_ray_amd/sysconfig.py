"""paddle.sysconfig (parity: python/paddle/sysconfig.py): include / lib dirs for building
custom native extensions against this framework (HIP kernel headers + runtime libs)."""
import os

_ROOT = os.path.dirname(os.path.abspath(__file__))


def get_include():
    return os.path.join(_ROOT, 'ops', 'csrc')


def get_lib():
    return os.path.join(_ROOT, 'ops')
