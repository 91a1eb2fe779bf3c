# qhuff_open order probes (diagnostic)
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ls-qpack_amd"))
mode = sys.argv[1] if len(sys.argv) > 1 else "a"
import qhuff
if mode == "b":
    import torch
for i in range(2):
    try:
        c = qhuff.Codec(0); print("open", i, "ok"); c.close()
    except Exception as e:
        print("open", i, "failed:", e)
import torch
print("torch", torch.cuda.device_count(), torch.cuda.is_available())
