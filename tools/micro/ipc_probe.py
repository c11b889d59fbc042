#!/usr/bin/env python3
"""Start the two sides of ``ipc_probe`` (tools/micro/ipc_probe.hip) as sibling
processes on GPU 0 and print both logs.  This launcher never touches the GPU.

    python tools/micro/ipc_probe.py [iters] [--cp-wait]
"""
import os
import subprocess
import sys
import time

here = os.path.dirname(os.path.abspath(__file__))
exe = os.path.join(here, "ipc_probe")
iters = next((a for a in sys.argv[1:] if a.isdigit()), "2000")
env = dict(os.environ)
env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
if "--cp-wait" in sys.argv:
    env["GPU_STREAMOPS_CP_WAIT"] = "1"
name = f"/sca_ipc_probe_{os.getpid()}"
a = subprocess.Popen([exe, "A", name, iters], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
time.sleep(0.2)
b = subprocess.Popen([exe, "B", name, iters], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
rc = 0
for tag, p in (("A", a), ("B", b)):
    try:
        out, _ = p.communicate(timeout=90)
    except subprocess.TimeoutExpired:
        p.kill()
        out, _ = p.communicate()
        out += f"\n{tag}: KILLED after 90 s\n"
    print(out, end="")
    print(f"[{tag} exit {p.returncode}]")
    rc = rc or p.returncode
try:
    os.unlink("/dev/shm" + name)
except OSError:
    pass
sys.exit(rc)
