"""AmdSmiBackend health-event logic against a fake ``amdsmi`` module (no GPU)."""
import sys
import types

from test_devices_sysfs import make_tree

from amdvgpu.plugin.devices import AmdSmiBackend


class _Evt:
    GPU_PRE_RESET = 1
    GPU_POST_RESET = 2
    RING_HANG = 4


def fake_amdsmi(events):
    m = types.ModuleType("amdsmi")
    handle = object()
    m.AmdSmiEvtNotificationType = _Evt
    m.amdsmi_init = lambda *a: None
    m.amdsmi_shut_down = lambda: None
    m.amdsmi_get_processor_handles = lambda: [handle]
    m.amdsmi_get_gpu_device_bdf = lambda h: "0000:05:00.0"
    m.amdsmi_get_gpu_asic_info = lambda h: {"market_name": "AMD Instinct MI355X"}
    m.amdsmi_init_gpu_event_notification = lambda h: None
    m.amdsmi_set_gpu_event_notification_mask = lambda h, mask: None
    m.amdsmi_get_gpu_event_notification = lambda timeout: [dict(e, processor_handle=handle) for e in events.pop(0)] \
        if events else []
    return m


def test_reset_events_drive_health(tmp_path, monkeypatch):
    kfd, drm = make_tree(tmp_path, ngpu=1)
    events = [[{"event": "AMDSMI_EVT_NOTIF_GPU_PRE_RESET"}], [{"event": "AMDSMI_EVT_NOTIF_GPU_POST_RESET"}],
              [{"event": "AMDSMI_EVT_NOTIF_VMFAULT"}]]
    monkeypatch.setitem(sys.modules, "amdsmi", fake_amdsmi(events))
    be = AmdSmiBackend(kfd_root=kfd, drm_root=drm)
    devs = be.devices()
    assert devs[0].product == "AMD Instinct MI355X"
    ev = be.poll_health(devs)
    assert [(e.uuid, e.healthy) for e in ev] == [(devs[0].uuid, False)]
    devs[0].healthy = False
    ev = be.poll_health(devs)
    assert any(e.healthy for e in ev)
    devs[0].healthy = True
    assert be.poll_health(devs) == []  # VM fault = application error, ignored
    be.close()
