"""The drop-in contract (SURVEY.md §8 b): every public function the backend
replaces keeps the reference's parameter names, order, kinds and defaults.

The reference signatures are data recorded from the reference modules by
tests/golden/make_signatures.py (tests/golden/signatures.json), so this test
runs anywhere.  Extensions of this backend are allowed only AFTER the
reference's parameters, as keyword parameters with a default."""

import inspect
import json
import os

import pytest

from conftest import GOLDEN

SIGS = json.load(open(os.path.join(GOLDEN, "signatures.json")))
OURS = {"get_isect_offsets": "isect_offset_encode"}  # the Triton wrapper's name for it


def _ours(name):
    import gsplat_hip
    from gsplat_hip import distributed
    n = OURS.get(name, name)
    mod = distributed if SIGS[name]["module"] == "gsplat.distributed" else gsplat_hip
    return getattr(mod, n)


@pytest.mark.parametrize("name", sorted(SIGS))
def test_signature_matches_reference(name):
    ref = SIGS[name]["params"]
    ours = list(inspect.signature(_ours(name)).parameters.values())
    assert len(ours) >= len(ref), (name, [p.name for p in ours])
    for (rname, rkind, rdef), p in zip(ref, ours):
        assert p.name == rname, (name, rname, p.name)
        assert p.kind.name == rkind, (name, rname, rkind, p.kind.name)
        ours_def = None if p.default is inspect.Parameter.empty else repr(p.default)
        assert ours_def == rdef, (name, rname, rdef, ours_def)
    for p in ours[len(ref):]:
        assert p.default is not inspect.Parameter.empty, (name, "extension without default",
                                                         p.name)
