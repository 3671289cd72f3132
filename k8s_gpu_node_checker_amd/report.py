"""Presentation: summary line, text table, JSON payload, Slack text.

Every user-facing string is byte-identical to the reference (SURVEY Appendix
A): the Korean summaries, ``⚠️`` as U+26A0 U+FE0F, the ``","`` breakdown
separator in the table versus ``", "`` in Slack, ``ljust`` column widths and
the ``json.dumps(ensure_ascii=False, indent=2)`` layout.

Rendering builds one string and writes it once instead of one ``print`` per
row (reference ``:240-249``); the bytes are the same.
"""

from __future__ import annotations

TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Dict, List, Optional, Sequence

SUMMARY_READY = "✅ Ready 상태의 GPU 노드: {ready}개 / 전체 GPU 노드: {total}개"
SUMMARY_NOT_READY = "⚠️ GPU 노드는 {total}개 있으나, Ready 상태 노드는 없습니다."
SUMMARY_NO_GPU = "❌ GPU 노드가 없습니다."
TABLE_EMPTY = "GPU 노드가 존재하지 않습니다."
SLACK_SENT = "✅ 슬랙 메시지를 성공적으로 전송했습니다."
SLACK_FAILED = "❌ 슬랙 메시지 전송에 실패했습니다."


def summary_line(gpu_nodes: Sequence[Dict], ready_gpu_nodes: Sequence[Dict]) -> str:
    """Reference ``:281-286``."""
    if ready_gpu_nodes:
        return SUMMARY_READY.format(ready=len(ready_gpu_nodes), total=len(gpu_nodes))
    if gpu_nodes:
        return SUMMARY_NOT_READY.format(total=len(gpu_nodes))
    return SUMMARY_NO_GPU


def _keys_str(breakdown: Dict[str, int], sep: str) -> str:
    return sep.join([f"{k}:{v}" for k, v in breakdown.items()])


def render_table(gpu_nodes: Sequence[Dict]) -> str:
    """Text table (reference ``print_table``, ``:229-249``), newline-terminated."""
    if not gpu_nodes:
        return TABLE_EMPTY + "\n"
    w_name = max(len("NAME"), max(len(n["name"]) for n in gpu_nodes))
    lines = [
        f"{'NAME'.ljust(w_name)}  READY  GPU(TOTAL)  GPU(KEYS)",
        f"{'-' * w_name}  -----  ----------  ---------",
    ]
    for n in gpu_nodes:
        bd = n["gpu_breakdown"]
        keys = _keys_str(bd, ",") if bd else "-"
        lines.append(f"{n['name'].ljust(w_name)}  {str(n['ready']).ljust(5)}  {str(n['gpus']).ljust(10)}  {keys}")
    lines.append("")
    return "\n".join(lines)


def render_text(gpu_nodes: Sequence[Dict], ready_gpu_nodes: Sequence[Dict]) -> str:
    return summary_line(gpu_nodes, ready_gpu_nodes) + "\n" + render_table(gpu_nodes)


def json_payload(gpu_nodes: List[Dict], ready_gpu_nodes: Sequence[Dict],
                 extra: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """Reference ``:274-278``: ``total_nodes`` counts GPU nodes only."""
    payload: Dict[str, Any] = {
        "total_nodes": len(gpu_nodes),
        "ready_nodes": len(ready_gpu_nodes),
        "nodes": gpu_nodes,
    }
    if extra:
        payload.update(extra)
    return payload


def render_json(payload: Dict[str, Any]) -> str:
    """``json.dumps(payload, ensure_ascii=False, indent=2)`` plus a newline.

    Uses the native emitter when it is built (byte-identical, checked by
    ``tests/test_fastpath.py``); the stdlib indent encoder is pure Python and
    is the dominant render cost at 1000 nodes.
    """
    from .ops import fastpath
    return fastpath.dumps_indent2(payload) + "\n"


def render_error_json(message: str) -> str:
    """Reference ``:322``: single line, no indent."""
    import json
    return json.dumps({"error": message}, ensure_ascii=False) + "\n"


def format_slack_message(gpu_nodes: Sequence[Dict], ready_gpu_nodes: Sequence[Dict],
                         health: Optional[Sequence[Optional[str]]] = None) -> str:
    """Slack text (reference ``format_slack_message``, ``:114-139``).

    ``health`` (optional, parallel to ``gpu_nodes``) appends the MI355X health
    verdict to each bullet; without it the text is byte-identical.
    """
    if ready_gpu_nodes:
        emoji = "✅"
        status = f"Ready 상태의 GPU 노드: {len(ready_gpu_nodes)}개 / 전체 GPU 노드: {len(gpu_nodes)}개"
    elif gpu_nodes:
        emoji = "⚠️"
        status = f"GPU 노드는 {len(gpu_nodes)}개 있으나, Ready 상태 노드는 없습니다."
    else:
        emoji = "❌"
        status = "GPU 노드가 없습니다."
    parts = [f"{emoji} *K8s GPU 노드 상태*\n{status}"]
    if gpu_nodes:
        parts.append("\n\n*노드 상세 정보:*")
        for i, n in enumerate(gpu_nodes):
            state = "✅ Ready" if n["ready"] else "❌ Not Ready"
            info = f"GPU: {n['gpus']}"
            if n["gpu_breakdown"]:
                info += f" ({_keys_str(n['gpu_breakdown'], ', ')})"
            line = f"\n• `{n['name']}`: {state}, {info}"
            if health is not None and i < len(health) and health[i]:
                line += f" [{health[i]}]"
            parts.append(line)
    return "".join(parts)
