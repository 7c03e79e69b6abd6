"""GPU OSD launches for one code (for rocprofv3 passes). usage: python tools/osd_once.py CODE COUNT"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as b  # noqa: E402

print(b.run_osd(sys.argv[1], int(sys.argv[2])))
