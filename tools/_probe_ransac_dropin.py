"""Probe: where the RANSAC drop-in's time goes (GPU box): the caller's state to words, the host replay of
CPython's draws (sv_ransac_draw), the draws + GPU evaluation (sv_ransac), and the whole drop-in call."""
import ctypes, os, random, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests")]
import numpy as np
import oracle
from svx import _abi, ransac
from test_prepass_cpu import carmask
disp, _ = oracle.synth_frame(0)
pts = np.ascontiguousarray(oracle.project(oracle.mask_disparity(disp, carmask()), None, 2)[0])
plist = list(pts)
n, k, trials = len(pts), 600, 600
sidx = np.empty((trials, k), np.int32); tri = np.empty((trials, 3), np.int32)
abc = np.empty((trials, 3)); err = np.empty(trials); flag = np.empty(trials, np.uint8); ran = ctypes.c_int(0)
random.seed(0)
st = random.getstate()
def t(name, fn, reps=20):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    print(f"{name:44s} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms", flush=True)
t("state -> words", lambda: np.array(st[1], dtype=np.uint32))
words = np.array(st[1], dtype=np.uint32)
def draw():
    w = words.copy()
    _abi.call("sv_ransac_draw", _abi.ptr(w), _abi.ptr(pts), n, 3, trials, k, _abi.ptr(sidx), _abi.ptr(tri), ctypes.byref(ran))
def full():
    w = words.copy()
    _abi.call("sv_ransac", _abi.ptr(w), _abi.ptr(pts), n, 3, trials, k, _abi.ptr(sidx), _abi.ptr(tri), _abi.ptr(abc),
              _abi.ptr(err), _abi.ptr(flag), ctypes.byref(ran))
t("sv_ransac_draw (host replay)", draw)
t("sv_ransac (replay + upload + eval + download)", full)
def dropin():
    random.setstate(st)
    ransac.RANSAC(plist, 600)
t("ransac.RANSAC (the drop-in, list of rows)", dropin)
def dropin_arr():
    random.setstate(st)
    ransac.RANSAC(pts, 600) if False else ransac.trials_gpu(pts, 600, st)
t("ransac.trials_gpu (array)", dropin_arr)
