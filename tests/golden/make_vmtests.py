"""Generate tests/golden/vmtests.json from the reference's VMTests fixtures.

Run in the build container (where /root/reference exists):
    python tests/golden/make_vmtests.py /root/reference/tests/laser/evm_testsuite/VMTests

The reference runs these official Ethereum VM known-answer tests through LASER
(tests/laser/evm_testsuite/evm_test.py:105-188, ignore list :33-60).  We keep the straight-line
ones — code built only from PUSH/DUP/SWAP/POP, arithmetic, comparison/bitwise, SHA3,
MLOAD/MSTORE/MSTORE8, SSTORE and STOP — as (code, pre-storage, post-storage) data; the tests
translate the code into tapes (tests/evm_translate.py) and check every stored value.  Only data
fields are copied: the test name, the bytecode and the storage maps.
"""
import json
import sys
from pathlib import Path

SUITES = [
    "vmArithmeticTest",
    "vmBitwiseLogicOperation",
    "vmSha3Test",
    "vmPushDupSwapTest",
    "vmIOandFlowOperations",
    "vmRandomTest",
    "vmTests",
]

# evm_test.py:33-60 ignore list (names only)
IGNORED = {
    "gas0", "gas1", "log1MemExp", "loop_stacklimit_1020", "loop_stacklimit_1021",
    "jumpTo1InstructionafterJump", "sstore_load_2", "jumpi_at_the_end",
}

SUPPORTED = set(range(0x01, 0x0C)) | set(range(0x10, 0x1E)) | {0x00, 0x20, 0x50, 0x51, 0x52,
                                                              0x53, 0x55}
SUPPORTED |= set(range(0x60, 0xA0))  # PUSH1..32, DUP1..16, SWAP1..16


def straight_line(code: bytes) -> bool:
    i = 0
    while i < len(code):
        op = code[i]
        if op not in SUPPORTED:
            return False
        if 0x60 <= op <= 0x7F:
            i += op - 0x5F
        i += 1
    return True


def main(root: str) -> None:
    out = []
    for suite in SUITES:
        for f in sorted((Path(root) / suite).glob("*.json")):
            data = json.loads(f.read_text())
            for name, t in data.items():
                if name in IGNORED or "post" not in t:
                    continue
                code = bytes.fromhex(t["exec"]["code"][2:])
                if not straight_line(code):
                    continue
                addr = t["exec"]["address"]
                pre = t["pre"].get(addr, {}).get("storage", {})
                post = t["post"].get(addr, {}).get("storage", {})
                out.append({
                    "suite": suite,
                    "name": name,
                    "code": code.hex(),
                    "pre_storage": pre,
                    "post_storage": post,
                })
    dst = Path(__file__).parent / "vmtests.json"
    dst.write_text(json.dumps(out, indent=0, sort_keys=True))
    print("wrote %d vectors to %s" % (len(out), dst))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else
         "/root/reference/tests/laser/evm_testsuite/VMTests")
