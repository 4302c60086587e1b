"""Which clock / power sources are readable on this box (bench.py's ClockSampler)."""
import glob
import os
import traceback

try:
    import amdsmi
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    print("amdsmi handles", len(hs))
    for h in hs[:2]:
        print(" bdf", amdsmi.amdsmi_get_gpu_device_bdf(h))
        print(" clk", amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.SYS))
        print(" pwr", amdsmi.amdsmi_get_power_info(h))
except Exception:
    traceback.print_exc()
for pat in ("/sys/class/drm/card*/device/pp_dpm_sclk", "/sys/class/drm/card*/device/hwmon/hwmon*/freq1_input",
            "/sys/class/drm/card*/device/hwmon/hwmon*/power1_average",
            "/sys/class/drm/card*/device/hwmon/hwmon*/power1_input",
            "/sys/class/drm/card*/device/gpu_metrics"):
    for f in glob.glob(pat)[:4]:
        try:
            data = open(f, "rb").read()
            print(f, len(data), data[:120])
        except Exception as e:
            print(f, "ERR", e)
print("HIP_VISIBLE_DEVICES", os.environ.get("HIP_VISIBLE_DEVICES"), os.environ.get("ROCR_VISIBLE_DEVICES"))
