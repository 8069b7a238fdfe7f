"""GPU image path (ops.image_decode, csrc/image_decode.hip) timing: a batch of 32 containers of
camera-like JPEGs (320x240 / 640x480, as tools/http_bench.py uploads) and of raw RGB8, graph-timed
alone and with 4 co-running copies."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    from test_image_decode import jpeg, photo

    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops.autotune import _time_multi
    from mlmicroservicetemplate_amd.plugins.builtin import image_container

    dev = torch.device("cuda:0")
    cases = {
        "jpeg320x240": [image_container(jpeg(photo(320, 240, seed=i), quality=90), "image/jpeg") for i in range(32)],
        "jpeg640x480": [image_container(jpeg(photo(640, 480, seed=i), quality=85), "image/jpeg") for i in range(32)],
        "raw224": [image_container(photo(224, 224, seed=i).tobytes(), "application/octet-stream") for i in range(32)],
    }
    for name, conts in cases.items():
        xs = [torch.from_numpy(np.stack(conts)).to(dev) for _ in range(4)]
        outs = [torch.empty(32, 224, 224, 3, device=dev, dtype=torch.uint8) for _ in range(4)]
        for c in (1, 4):
            ms = _time_multi([lambda i=i: ops.image_decode(xs[i], out=outs[i]) for i in range(c)], iters=20)
            print(json.dumps({"case": name, "batch": 32, "conc": c, "us_per_batch": round(ms * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
