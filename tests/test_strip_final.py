"""Final strip semantics, python oracle and native C++."""
import pytest

from quorum_amd.ops import native
from quorum_amd.ops.reference import strip_thinking_tags

TAGS = ["think", "reason", "reasoning", "thought"]
CASES = [
    ("<think>x</reason>Y", "<think>x</reason>Y"),
    ("<think>a<think>b</think>c</think>D", "c</think>D"),
    ("<think>unclosed Y", "<think>unclosed Y"),
    ("<THINK>x</think>Y", "Y"),
    ("  <think>x</think>  Y  ", "Y"),
    ("<think>a<reason>b</reason>", "<think>a"),
    ("pre<reasoning>r</reasoning>post<thought>t\n\nt</thought>!", "prepost!"),
    ("　  text  ", "text"),
    ("", ""),
    ("<think></think>", ""),
    ("a<think>1</think>b<think>2</think>c", "abc"),
]


def _impls():
    out = [("python", lambda t, tags: strip_thinking_tags(t, tags))]
    if native.available():
        out.append(("native", lambda t, tags: native.strip_fn(tags)(t, True)))
    return out


@pytest.mark.parametrize("impl", _impls(), ids=lambda p: p[0])
@pytest.mark.parametrize("text,expected", CASES)
def test_strip(impl, text, expected):
    assert impl[1](text, TAGS) == expected


def test_disabled_is_identity():
    assert strip_thinking_tags("  <think>x</think> ", TAGS, hide_intermediate=False) == "  <think>x</think> "
