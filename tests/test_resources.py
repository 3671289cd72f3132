"""R1/R2: registry order and bug-compatible quantity parsing (reference check-gpu-node.py:39-44, :181-196)."""
from hypothesis import given, strategies as st

from k8s_gpu_node_checker_amd.models.resources import (GPU_RESOURCE_KEYS, PRIMARY_GPU_KEY, gpu_breakdown,
                                                       parse_gpu_quantity, quantity_text)


def test_registry_order_is_output_order():
    assert GPU_RESOURCE_KEYS == ("nvidia.com/gpu", "amd.com/gpu", "gpu.intel.com/i915", "intel.com/gpu")
    assert PRIMARY_GPU_KEY == "amd.com/gpu"


def test_zero_is_kept_missing_and_empty_are_skipped():
    assert parse_gpu_quantity("0") == 0
    assert parse_gpu_quantity(0) == 0          # the k8s client str()s numbers: "0" is kept
    assert parse_gpu_quantity(None) is None
    assert parse_gpu_quantity("") is None


def test_non_integer_quantities_are_dropped():
    for v in ("1k", "500m", "8.0", "1e3", "Infinity", "eight", " ", True, 8.0, [], {}):
        assert parse_gpu_quantity(v) is None, v


def test_python_int_semantics():
    assert parse_gpu_quantity(" 8 ") == 8
    assert parse_gpu_quantity("+8") == 8
    assert parse_gpu_quantity("-2") == -2
    assert parse_gpu_quantity("0008") == 8
    assert parse_gpu_quantity("1_000") == 1000
    assert parse_gpu_quantity("８") == 8  # fullwidth digit: int() accepts it


def test_breakdown_follows_registry_order_not_capacity_order():
    cap = {"intel.com/gpu": "1", "gpu.intel.com/i915": "2", "amd.com/gpu": "3", "nvidia.com/gpu": "4", "cpu": "8"}
    assert list(gpu_breakdown(cap)) == list(GPU_RESOURCE_KEYS)


def test_breakdown_of_missing_capacity():
    assert gpu_breakdown(None) == {}
    assert gpu_breakdown({}) == {}
    assert gpu_breakdown("not a map") == {}


@given(st.text(max_size=12))
def test_quantity_matches_reference_expression(s):
    # the reference: `if not val: continue; try: int(str(val)) except: pass`
    try:
        expect = int(str(s)) if s else None
    except Exception:
        expect = None
    assert parse_gpu_quantity(s) == expect


@given(st.one_of(st.integers(), st.booleans(), st.none(), st.floats(allow_nan=False)))
def test_quantity_of_json_scalars(v):
    text = quantity_text(v)
    if v is None:
        assert text is None
    else:
        assert text == str(v)
