#!/usr/bin/env python3
"""Development timing (not shipped, not a test): the rowpass alone and the
in-graph minibatch step at H 256, mb 4096, for the current SATRL_RP_DUAL
setting (run once with 0 and once with 1)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for dual in ("0", "1"):
    env = dict(os.environ, SATRL_RP_DUAL=dual)
    for tool in ("rowpass_ab.py", "minibatch_time.py"):
        args = [sys.executable, os.path.join(ROOT, "tools", tool)] + (["4096", "512"] if tool.startswith("mini") else [])
        out = subprocess.run(args, env=env, capture_output=True, text=True, timeout=300)
        print(f"SATRL_RP_DUAL={dual} {tool}:\n{out.stdout}{out.stderr[-2000:] if out.returncode else ''}", flush=True)
