#!/usr/bin/env python3
"""Which combination of the native libraries aborts at interpreter exit?  Each variant runs in its own
child process; the run stops at the first child that does not exit 0 (one abnormal exit per call)."""
import subprocess
import sys

VARIANTS = {
    "fabric": "F()",
    "probe-close-fabric": "P(); close(); F()",
    "torch-rccl": "T()",
    "probe-torch-rccl": "P(); T()",
    "probe-fabric-close": "P(); F(); close()",
    "fabric-probe": "F(); P()",
    "probe-fabric": "P(); F()",
    "probe-diag-fabric": "P(); D(); F()",
    "torch-rccl-probe": "T(); P()",
    "soak-order": "D(); F(); P(); F(); P(); D()",
    "bench-order": "import torch; P(); D(); T()",
}
PRE = ("import sys; sys.path.insert(0, '.')\n"
       "from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag, fabric\n"
       "P = lambda: amdsmi_probe.probe_native('x')\n"
       "F = lambda: fabric.collective_suite([0], sizes=[1 << 20], iters=1, warmup=0)\n"
       "D = lambda: diag.hbm(0, gib=0.5, iters=1)\n"
       "close = lambda: amdsmi_probe.close()\n"
       "def T():\n"
       "    import os, torch, torch.distributed as dist\n"
       "    os.environ.update(RANK='0', WORLD_SIZE='1', MASTER_ADDR='127.0.0.1', MASTER_PORT='29611')\n"
       "    torch.cuda.set_device(0)\n"
       "    dist.init_process_group('nccl', device_id=torch.device('cuda:0'))\n"
       "    t = torch.ones(1 << 20, device='cuda:0'); dist.all_reduce(t); torch.cuda.synchronize()\n"
       "    dist.destroy_process_group()\n")
for name in (sys.argv[1:] or VARIANTS):
    p = subprocess.run([sys.executable, "-X", "faulthandler", "-c", PRE + VARIANTS[name]], capture_output=True, text=True, timeout=120)
    print(name, p.returncode, "\n".join(p.stderr.strip().splitlines()[-25:]), flush=True)
    if p.returncode != 0:
        break
