"""Run the configs[1] forward back-to-back for a few seconds while sampling the
GPU's clock and power with rocm-smi in a child process: tells whether the
forward is power/clock-capped (DVFS) or issue-bound at full clock.
Usage: python tools/exp/clock_probe.py [seconds]"""
import os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch
import fa_hip

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
N, d, BH = int(os.environ.get("FA_N", 4096)), int(os.environ.get("FA_D", 64)), int(os.environ.get("FA_BH", 64))
g = torch.Generator(device="cuda").manual_seed(0)
Q, K, V = [fa_hip.jl_empty((N, d, BH), torch.bfloat16) for _ in range(3)]
for t in (Q, K, V):
    t.copy_(torch.randn((N, d, BH), generator=g, device="cuda"))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))


def smi():
    try:
        return subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--showtemp"],
                              capture_output=True, text=True, timeout=20).stdout
    except Exception as e:  # noqa: BLE001
        return f"rocm-smi failed: {e}"


print("== idle\n" + smi(), flush=True)
t_end = time.time() + secs
n = 0
e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
e0.record()
probe_at = time.time() + secs / 2
probed = False
while time.time() < t_end:
    for _ in range(50):
        fa_hip.dense_fa_(O, l, m, Q, K, V)
    n += 50
    if not probed and time.time() > probe_at:
        probed = True
        proc = subprocess.Popen(["rocm-smi", "--showpower", "--showclocks", "--showtemp"],
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
e1.record(); torch.cuda.synchronize()
print("== under load\n" + proc.communicate(timeout=60)[0], flush=True)
t = e0.elapsed_time(e1) / 1e3 / n
print(f"{n} launches, {t*1e6:.1f} us each, {4.0*BH*N*N*d/t/1e12:.1f} TFLOP/s", flush=True)
