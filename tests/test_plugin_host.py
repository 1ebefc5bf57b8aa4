"""CPU: host-side logic of the plugin/common mirror that needs no device (plugin/plugin_test.go
TestSorter/TestMock, common/common_test.go payload slicing, encryption gating)."""
from quantum_amd import common, plugin


def test_constants():
    # common/common.go:16-38
    assert (common.IPStart, common.IPEnd, common.PacketStart, common.HeaderSize) == (0, 4, 4, 4)
    assert common.MaxPacketLength == 1472 and common.OverflowSize == 35 and common.MTU == 1433
    # sealed MTU packet fits the Raw buffer: 4 + 1433 + 28 <= 1472
    assert common.HeaderSize + common.MTU + 28 <= common.MaxPacketLength


def test_payload_slicing():
    """common/common_test.go:502-530 on its 6-byte fixture shape."""
    raw = bytearray([1, 2, 3, 4, 5, 6])
    p = common.NewTunPayload(raw, 2)
    assert p.IPAddress.tobytes() == bytes([1, 2, 3, 4]) and p.Packet.tobytes() == bytes([5, 6]) and p.Length == 6
    s = common.NewSockPayload(raw, 6)
    assert s.IPAddress.tobytes() == bytes([1, 2, 3, 4]) and s.Packet.tobytes() == bytes([5, 6]) and s.Length == 6


def test_sorter_orders():
    """plugin/plugin_test.go:58-87: outgoing ascending, incoming reversed."""
    enc, _ = plugin.New(plugin.EncryptionPlugin)
    mock, _ = plugin.New(plugin.MockPlugin)
    assert [p.Order() for p in plugin.Sorter([mock, enc])] == [1, 2]
    assert [p.Name() for p in plugin.Sorter([enc, mock], reverse=True)] == ["mock", "encryption"]
    assert plugin.Incoming == 0 and plugin.Outgoing == 1
    assert (plugin.CompressionPluginOrder, plugin.EncryptionPluginOrder, plugin.MockPluginOrder) == (0, 1, 2)


def test_mock():
    """plugin/plugin_test.go:218-232."""
    mock, _ = plugin.New(plugin.MockPlugin)
    assert mock.Apply(plugin.Outgoing, None, None) == (None, None, True)
    assert mock.Close() is None and mock.Order() == plugin.MockPluginOrder


def test_new_unknown():
    p, err = plugin.New("nope")
    assert p is None and err is not None


def test_encryption_passthrough_when_peer_lacks_plugin():
    """plugin/encryption.go:17-19: no device work, packet untouched, ok."""
    enc, _ = plugin.New(plugin.EncryptionPlugin)
    raw = bytearray(range(64))
    p = common.NewTunPayload(raw, 40)
    m = common.Mapping(SupportedPlugins=["compression"], AES=None)
    for d in (plugin.Incoming, plugin.Outgoing):
        out, mm, ok = enc.Apply(d, p, m)
        assert ok and out is p and mm is m and raw == bytearray(range(64)) and out.Length == 44
    assert enc.Name() == "encryption" and enc.Order() == 1
