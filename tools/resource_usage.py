"""Print per-kernel VGPRs / scratch / occupancy / LDS of one source file (dev tool):
  python tools/resource_usage.py viso_amd/csrc/direct.hip [-DFLAG ...]"""
import os
sys_path_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import sys
sys.path.insert(0, sys_path_root)
import subprocess
import viso_amd.build as b
flags=b.COMMON+sys.argv[2:]
cmd=[b.HIPCC]+flags+['-c',sys.argv[1],'-o','/tmp/ru.o','-Rpass-analysis=kernel-resource-usage']
r=subprocess.run(cmd,capture_output=True,text=True)
blocks=r.stderr.split('Function Name: ')
for bl in blocks[1:]:
    name=bl.split('\n')[0]
    keep=[l.split('remark: ')[-1].split(' [-R')[0].strip() for l in bl.split('\n') if any(k in l for k in ('VGPRs:','ScratchSize','Occupancy','LDS Size'))]
    print(name[:70], keep)
