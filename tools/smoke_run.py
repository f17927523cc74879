#!/usr/bin/env python3
"""__graft_entry__.smoke() as a script (for tools/gpu_session.sh py:tools/smoke_run.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.smoke()
print("smoke ok")
