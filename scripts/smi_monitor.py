"""Sample GPU power / clocks / activity every 0.5 s (amdsmi bindings) into a JSONL file
until killed: run in the background next to a benchmark to see whether it runs at
the power cap (clock throttling shows up as a falling gfx clock)."""
import json
import os
import sys
import time

sys.path.append("/opt/rocm/share/amd_smi")
import amdsmi  # noqa: E402

out = open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/smi.jsonl", "w")
amdsmi.amdsmi_init()
h = amdsmi.amdsmi_get_processor_handles()[0]
t0 = time.time()
while True:
    d = {"t": round(time.time() - t0, 2)}
    for name, fn in (("power", lambda: amdsmi.amdsmi_get_power_info(h)),
                     ("gfx_clk", lambda: amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)),
                     ("mem_clk", lambda: amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.MEM)),
                     ("act", lambda: amdsmi.amdsmi_get_gpu_activity(h)),
                     ("temp", lambda: amdsmi.amdsmi_get_temp_metric(h, amdsmi.AmdSmiTemperatureType.HOTSPOT,
                                                                    amdsmi.AmdSmiTemperatureMetric.CURRENT))):
        try:
            d[name] = fn()
        except Exception as e:  # noqa: BLE001
            d[name] = f"err {type(e).__name__}"
    out.write(json.dumps(d, default=str) + "\n")
    out.flush()
    time.sleep(0.5)
