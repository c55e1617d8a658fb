import json, os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oxidized-neural-orchestra_amd"))
import torch, ono_amd, bench
r = bench.sparse_codec(torch, ono_amd)
print(json.dumps(r)[:3000])
