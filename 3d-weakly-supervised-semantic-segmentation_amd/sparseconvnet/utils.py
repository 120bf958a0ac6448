"""Checkpoint helpers with SCN's naming and pruning contract.

train.py:37 calls `checkpoint_restore(model, exp_name, 'model', use_cuda)` and
expects the next epoch back; train.py:91 calls
`checkpoint_save(model, exp_name, 'model', epoch, use_cuda)`.  Files are
`<exp_name>-%09d-<name2>.pth`; saving epoch e removes epoch e-1's file unless
e-1 is a power of two.  Loading uses weights_only=True.
"""
from __future__ import annotations

import glob
import os

import torch


def is_power2(num):
    num = int(num)
    return num != 0 and (num & (num - 1)) == 0


def _fname(exp_name, epoch, name2):
    return f"{exp_name}-{int(epoch):09d}-{name2}.pth"


def checkpoint_save(model, exp_name, name2, epoch, use_cuda=True):
    f = _fname(exp_name, epoch, name2)
    model.cpu()
    torch.save(model.state_dict(), f)
    if use_cuda:
        model.cuda()
    prev = _fname(exp_name, int(epoch) - 1, name2)
    if os.path.isfile(prev) and not is_power2(int(epoch) - 1):
        os.remove(prev)


def checkpoint_restore(model, exp_name, name2, use_cuda=True, epoch=0):
    if use_cuda:
        model.cpu()
    if epoch > 0:
        f = _fname(exp_name, epoch, name2)
        if not os.path.isfile(f):
            raise FileNotFoundError(f)
        model.load_state_dict(torch.load(f, map_location="cpu", weights_only=True))
    else:
        files = sorted(glob.glob(f"{glob.escape(exp_name)}-*-{glob.escape(name2)}.pth"))
        if files:
            f = files[-1]
            model.load_state_dict(torch.load(f, map_location="cpu", weights_only=True))
            epoch = int(f[len(exp_name) + 1:-len(name2) - 5])
    if use_cuda:
        model.cuda()
    return epoch + 1
