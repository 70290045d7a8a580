import json, os, subprocess
out = {}
def sh(c):
    try: return subprocess.run(c, shell=True, capture_output=True, text=True, timeout=60).stdout[-4000:]
    except Exception as e: return repr(e)
out["id"] = sh("id"); out["ld_preload_env"] = os.environ.get("LD_PRELOAD"); out["ld_so_preload"] = sh("cat /etc/ld.so.preload")
out["dev"] = sh("ls -la /dev/dri /dev/kfd"); out["kfd_proc"] = sh("ls -la /sys/class/kfd/kfd/proc | head; ls /sys/class/kfd/kfd/proc/*/ 2>&1 | head -30")
out["kfd_nodes"] = sh("for n in /sys/class/kfd/kfd/topology/nodes/*; do echo $n; cat $n/name; grep -E 'simd_count|gpu_id|unique_id|location_id|drm_render_minor|num_xcc|cu_per_simd|array_count|simd_arrays|max_engine|domain' $n/properties; done")
out["drm_busy"] = sh("cat /sys/class/drm/card*/device/gpu_busy_percent; ls /sys/class/drm/")
out["lspci"] = sh("lspci 2>&1 | head -20")
try:
    import amdsmi
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    out["amdsmi_n"] = len(hs)
    devs = []
    for h in hs:
        d = {}
        for name, fn in [("uuid", lambda: amdsmi.amdsmi_get_gpu_device_uuid(h)),
                         ("bdf", lambda: amdsmi.amdsmi_get_gpu_device_bdf(h)),
                         ("asic", lambda: amdsmi.amdsmi_get_gpu_asic_info(h)),
                         ("vram_total", lambda: amdsmi.amdsmi_get_gpu_memory_total(h, amdsmi.AmdSmiMemoryType.VRAM)),
                         ("vram_usage", lambda: amdsmi.amdsmi_get_gpu_memory_usage(h, amdsmi.AmdSmiMemoryType.VRAM)),
                         ("compute_partition", lambda: amdsmi.amdsmi_get_gpu_compute_partition(h)),
                         ("memory_partition", lambda: amdsmi.amdsmi_get_gpu_memory_partition(h)),
                         ("activity", lambda: amdsmi.amdsmi_get_gpu_activity(h)),
                         ("kfd", lambda: amdsmi.amdsmi_get_gpu_kfd_info(h)),
                         ("enum", lambda: amdsmi.amdsmi_get_gpu_enumeration_info(h)),
                         ("numa", lambda: amdsmi.amdsmi_topo_get_numa_node_number(h)),
                         ("procs", lambda: amdsmi.amdsmi_get_gpu_process_list(h)),
                         ("ecc", lambda: amdsmi.amdsmi_get_gpu_total_ecc_count(h)),
                         ("xgmi", lambda: amdsmi.amdsmi_get_xgmi_info(h)),
                         ]:
            try: d[name] = str(fn())
            except Exception as e: d[name] = "ERR " + repr(e)
        devs.append(d)
    out["amdsmi"] = devs
    out["amdsmi_funcs"] = [f for f in dir(amdsmi) if f.startswith("amdsmi_")]
except Exception as e:
    out["amdsmi_err"] = repr(e)
print(json.dumps(out, indent=1))
