"""Does an event query from ANOTHER thread invalidate a global-mode capture on this image?
(the hypothesis behind the watchdog's relaxed capture mode). Prints one line per mode."""
import threading
import time

import torch

from tutorial_torch_distributed_data_parallel_amd._native import native


def trial() -> str:
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        native().debug_spin_ms(1000)
        ev = torch.cuda.Event()
        ev.record(side)
    stop = threading.Event()

    def poll():
        while not stop.is_set():
            ev.query()
            time.sleep(0.02)

    t = threading.Thread(target=poll)
    t.start()
    x = torch.ones(1024, device="cuda")
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode="global"):
            y = x * 2
            time.sleep(0.3)
        res = "capture ok"
    except Exception as e:  # noqa: BLE001
        res = f"capture FAILED: {str(e).splitlines()[0]}"
    stop.set()
    t.join()
    torch.cuda.synchronize()
    return res


print("python thread polling hipEventQuery during a global capture:", trial(), flush=True)
