"""Clock / power / temperature readings of the GPU a process runs on (bench provenance).

The same code measures a few percent apart on different MI355X boxes (profiles/README r4e:
285.7-300.1 MH/s); the bench line carries these readings from its start and end so a
difference can be put on the box (clocks, power capping, temperature) or on the code. Read-only
queries through amdsmi (ROCm SMI library); every key is simply absent when amdsmi, a field or
the device is unavailable (CPU rehearsals, containers without the driver).

Reference metric surface: the reference reports mining state through getmininginfo
(/root/reference/src/rpc/mining.cpp:209-250); it has no device telemetry.
"""
from __future__ import annotations

_STATE: dict = {}


def _handle(device_index: int):
    """amdsmi handle of torch's cuda:<device_index>, matched by PCI bus (amdsmi enumerates every
    GPU of the machine, not only the visible ones)."""
    key = ("h", device_index)
    if key in _STATE:
        return _STATE[key]
    import amdsmi
    import torch

    if not _STATE.get("init"):
        amdsmi.amdsmi_init()
        _STATE["init"] = True
    props = torch.cuda.get_device_properties(device_index)
    want = (int(getattr(props, "pci_domain_id", 0)), int(props.pci_bus_id), int(props.pci_device_id))
    found = None
    for h in amdsmi.amdsmi_get_processor_handles():
        bdf = str(amdsmi.amdsmi_get_gpu_device_bdf(h))  # "0000:05:00.0"
        dom, bus, rest = bdf.split(":")
        dev = rest.split(".")[0]
        if (int(dom, 16), int(bus, 16), int(dev, 16)) == want:
            found = h
            break
    _STATE[key] = found
    return found


def snapshot(device_index: int = 0) -> dict:
    """{sclk_mhz, mclk_mhz, power_w, temp_hotspot_c, temp_hbm_c, gfx_activity_pct} for the device
    (a subset, or {}, when something is unavailable)."""
    out: dict = {}
    try:
        import amdsmi

        h = _handle(device_index)
        if h is None:
            return out
    except Exception:
        return out
    try:
        m = amdsmi.amdsmi_get_gpu_metrics_info(h)

        def num(k):
            v = m.get(k)
            return v if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF) else None

        for src, dst in (("current_gfxclk", "sclk_mhz"), ("average_gfxclk_frequency", "sclk_avg_mhz"),
                         ("current_uclk", "mclk_mhz"), ("current_socket_power", "power_w"),
                         ("average_socket_power", "power_avg_w"), ("temperature_hotspot", "temp_hotspot_c"),
                         ("temperature_mem", "temp_hbm_c"), ("average_gfx_activity", "gfx_activity_pct")):
            v = num(src)
            if v is not None:
                out[dst] = v
    except Exception:
        pass
    try:
        if "sclk_mhz" not in out:
            out["sclk_mhz"] = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)["clk"]
        if "mclk_mhz" not in out:
            out["mclk_mhz"] = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.MEM)["clk"]
    except Exception:
        pass
    try:
        if "power_w" not in out:
            p = amdsmi.amdsmi_get_power_info(h)
            v = p.get("current_socket_power") or p.get("average_socket_power")
            if isinstance(v, (int, float)):
                out["power_w"] = v
    except Exception:
        pass
    try:
        if "temp_hotspot_c" not in out:
            out["temp_hotspot_c"] = amdsmi.amdsmi_get_temp_metric(h, amdsmi.AmdSmiTemperatureType.HOTSPOT,
                                                                  amdsmi.AmdSmiTemperatureMetric.CURRENT)
    except Exception:
        pass
    return out
