import sys, os
order = sys.argv[1]
sys.path.insert(0, "divortio-lz4_amd")
if order == "torch_first":
    import torch
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
    import lz4mi
    print("lz4mi init", lz4mi.lib().lz4mi_init(0))
else:
    import lz4mi
    print("lz4mi init", lz4mi.lib().lz4mi_init(0))
    import torch
    print("torch avail", torch.cuda.is_available())
print(open("/proc/self/maps").read().count("libamdhip64"), [l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l][:1])
