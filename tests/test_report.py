"""R10/R12/R14: byte-exact rendering against SURVEY Appendix A."""
import json

from k8s_gpu_node_checker_amd import report
from k8s_gpu_node_checker_amd.models.node import scan_items
from k8s_gpu_node_checker_amd.testing import fixtures

A1 = """✅ Ready 상태의 GPU 노드: 2개 / 전체 GPU 노드: 2개
NAME        READY  GPU(TOTAL)  GPU(KEYS)
----------  -----  ----------  ---------
gpu-node-1  True   4           nvidia.com/gpu:4
gpu-node-2  True   8           nvidia.com/gpu:8
"""

A3_NOGPU = "❌ GPU 노드가 없습니다.\nGPU 노드가 존재하지 않습니다.\n"

A3_NOTREADY = """⚠️ GPU 노드는 2개 있으나, Ready 상태 노드는 없습니다.
NAME   READY  GPU(TOTAL)  GPU(KEYS)
-----  -----  ----------  ---------
gpu-a  False  8           amd.com/gpu:8
gpu-b  False  8           amd.com/gpu:8
"""

A4 = """✅ Ready 상태의 GPU 노드: 3개 / 전체 GPU 노드: 4개
NAME                              READY  GPU(TOTAL)  GPU(KEYS)
--------------------------------  -----  ----------  ---------
zero-and-amd                      True   8           nvidia.com/gpu:0,amd.com/gpu:8
weird-qty                         True   2           intel.com/gpu:2
mixed-all-keys                    True   10          nvidia.com/gpu:4,amd.com/gpu:3,gpu.intel.com/i915:2,intel.com/gpu:1
a-very-long-node-name-0123456789  False  8           amd.com/gpu:8
"""

A5_READY = ("✅ *K8s GPU 노드 상태*\nReady 상태의 GPU 노드: 2개 / 전체 GPU 노드: 2개\n\n*노드 상세 정보:*\n"
            "• `gpu-node-1`: ✅ Ready, GPU: 4 (nvidia.com/gpu:4)\n• `gpu-node-2`: ✅ Ready, GPU: 8 (nvidia.com/gpu:8)")


def scan(name):
    return scan_items(fixtures.golden(name))


def test_text_readme():
    s = scan("readme")
    assert report.render_text(s.gpu_nodes, s.ready_gpu_nodes) == A1


def test_text_nogpu_and_notready():
    s = scan("nogpu")
    assert report.render_text(s.gpu_nodes, s.ready_gpu_nodes) == A3_NOGPU
    s = scan("notready")
    assert report.render_text(s.gpu_nodes, s.ready_gpu_nodes) == A3_NOTREADY
    assert "⚠️" in A3_NOTREADY


def test_text_edge():
    s = scan("edge")
    assert report.render_text(s.gpu_nodes, s.ready_gpu_nodes) == A4


def test_json_matches_stdlib_layout():
    for g in fixtures.GOLDEN:
        s = scan(g)
        p = report.json_payload(s.gpu_nodes, s.ready_gpu_nodes)
        assert report.render_json(p) == json.dumps(p, ensure_ascii=False, indent=2) + "\n"


def test_json_edge_details():
    s = scan("edge")
    doc = json.loads(report.render_json(report.json_payload(s.gpu_nodes, s.ready_gpu_nodes)))
    assert doc["total_nodes"] == 4 and doc["ready_nodes"] == 3
    mixed = [n for n in doc["nodes"] if n["name"] == "mixed-all-keys"][0]
    assert mixed["taints"] == [{"key": "amd.com/gpu", "value": None, "effect": "NoSchedule"},
                               {"key": "dedicated", "value": "ml", "effect": "NoExecute"}]
    weird = [n for n in doc["nodes"] if n["name"] == "weird-qty"][0]
    assert weird["labels"] == {"k": "한글"}
    assert '"k": "한글"' in report.render_json(report.json_payload(s.gpu_nodes, s.ready_gpu_nodes))
    assert doc["nodes"][0]["gpu_breakdown"] == {"nvidia.com/gpu": 0, "amd.com/gpu": 8}


def test_nometa_node():
    s = scan("nometa")
    assert s.gpu_nodes[0]["name"] == "" and s.gpu_nodes[0]["labels"] == {}


def test_slack_texts():
    s = scan("readme")
    assert report.format_slack_message(s.gpu_nodes, s.ready_gpu_nodes) == A5_READY
    s = scan("notready")
    assert report.format_slack_message(s.gpu_nodes, s.ready_gpu_nodes).startswith(
        "⚠️ *K8s GPU 노드 상태*\nGPU 노드는 2개 있으나, Ready 상태 노드는 없습니다.\n\n*노드 상세 정보:*\n"
        "• `gpu-a`: ❌ Not Ready, GPU: 8 (amd.com/gpu:8)")
    assert report.format_slack_message([], []) == "❌ *K8s GPU 노드 상태*\nGPU 노드가 없습니다."
    s = scan("edge")
    assert "GPU: 8 (nvidia.com/gpu:0, amd.com/gpu:8)" in report.format_slack_message(s.gpu_nodes, s.ready_gpu_nodes)


def test_slack_health_notes_are_opt_in():
    s = scan("readme")
    txt = report.format_slack_message(s.gpu_nodes, s.ready_gpu_nodes, ["MI355X 8/8 healthy", None])
    assert "• `gpu-node-1`: ✅ Ready, GPU: 4 (nvidia.com/gpu:4) [MI355X 8/8 healthy]" in txt
    assert txt.endswith("• `gpu-node-2`: ✅ Ready, GPU: 8 (nvidia.com/gpu:8)")


def test_slack_payload_bytes():
    from k8s_gpu_node_checker_amd.notify.slack import slack_payload
    s = scan("readme")
    body = slack_payload(report.format_slack_message(s.gpu_nodes, s.ready_gpu_nodes), "GPU-Monitor")
    assert len(body) == 373  # Appendix A.5 Content-Length
    assert list(json.loads(body)) == ["text", "username", "icon_emoji"]
    assert body.isascii()


def test_error_json_is_single_line():
    assert report.render_error_json("(403)\nReason: Forbidden\n") == '{"error": "(403)\\nReason: Forbidden\\n"}\n'
