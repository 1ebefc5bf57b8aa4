"""What GPU telemetry this box exposes to an unprivileged process (record the
clock and power behind every headline).  Prints amdsmi's metrics for the device torch sees as cuda:0,
its power cap, and the hwmon files of that PCI device, as JSON lines.  Run on the GPU box."""
import glob
import json
import os
import sys


def main() -> None:
    import torch

    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    print(json.dumps({"torch_bdf": bdf, "name": p.name}))
    dev = f"/sys/bus/pci/devices/{bdf}"
    files = {}
    for f in sorted(glob.glob(dev + "/hwmon/hwmon*/*")) + [dev + "/gpu_metrics", dev + "/pp_dpm_sclk",
                                                           dev + "/power_dpm_force_performance_level"]:
        try:
            v = open(f, "rb").read()
            files[os.path.basename(f)] = v[:200].decode("latin1").strip() if not f.endswith("gpu_metrics") else len(v)
        except OSError as e:
            files[os.path.basename(f)] = f"ERR {e.errno}"
    print(json.dumps({"sysfs": files}))
    try:
        import amdsmi
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"amdsmi_import": repr(e)}))
        return
    try:
        amdsmi.amdsmi_init()
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"amdsmi_init": repr(e)}))
        return
    hs = amdsmi.amdsmi_get_processor_handles()
    print(json.dumps({"handles": len(hs), "bdfs": [amdsmi.amdsmi_get_gpu_device_bdf(h) for h in hs]}))
    for h in hs:
        if amdsmi.amdsmi_get_gpu_device_bdf(h).lower() != bdf.lower():
            continue
        for name, fn in (("metrics", lambda: amdsmi.amdsmi_get_gpu_metrics_info(h)),
                         ("power_info", lambda: amdsmi.amdsmi_get_power_info(h)),
                         ("power_cap", lambda: amdsmi.amdsmi_get_power_cap_info(h)),
                         ("clock_gfx", lambda: amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)),
                         ("activity", lambda: amdsmi.amdsmi_get_gpu_activity(h))):
            try:
                v = fn()
                print(json.dumps({name: v}, default=str))
            except Exception as e:  # noqa: BLE001
                print(json.dumps({name: repr(e)}))
    amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    sys.exit(main())
