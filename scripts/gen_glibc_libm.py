#!/usr/bin/env python3
"""Generate csrc/vpt_glibc.h: the eight libm functions on the tracer's path, bit-identical to the
glibc the reference links on x86-64 hosts with FMA + AVX2.

Why: the reference (src/rt.cpp, include/*.h) calls libm's exp/log/sin/cos/tan/atan/atan2/acos
(include/vptSamplingFunctions.h:11-62, include/samplingFunctions.h:47-82,
include/microFacetUtilities.h:34-84, include/volumetricBasicFunctions.h:14-21,209-223) and
several branches of its estimators flip on the last bit of those results.  Per-
channel RMSE < 1e-4 against the reference's own images therefore needs the reference's libm, bit
for bit, on the GPU.  glibc 2.35 selects its FMA variants at load time (ifunc: FMA && AVX2 usable
-- true on the container's Xeon and on the GPU box's EPYC hosts), so this script translates THOSE
machine-code bodies -- not the generic C sources, whose rounding differs wherever the FMA build
contracted a*b+c -- into portable C that the HIP kernel and the oracle compile alike.

How: `objdump -d` of the pinned libm.so.6 (build-id checked below); every reachable instruction of
each function becomes one C statement over 64-bit register variables (x86 scalar-double semantics:
IEEE +-*/ and fused multiply-add, comisd flags, integer flags), rip-relative constants become
literals, table lookups read `gl_tab`, an extract of the library's read-only tables.  The mxcsr
save/restore (rounding mode is round-to-nearest on both sides), the stack protector and errno writes
are dropped; calls into the huge-argument reduction (__branred, |x| >= 105414350, never reached by
the tracer's angles) return NaN.  tests/test_glibc_libm.py checks the result against the host's
libm bit for bit on tens of millions of arguments per function.

Usage: python3 scripts/gen_glibc_libm.py [--libm /lib/x86_64-linux-gnu/libm.so.6]
"""
import argparse
import os
import re
import struct
import subprocess
import sys

BUILD_ID = "df46fc5774ae8aaaf6efcb97dc7b91532056b898"   # Ubuntu GLIBC 2.35-0ubuntu3.12
# FMA-variant entry points (resolved from the ifunc resolvers of exp/log/sin/cos/tan/atan and the
# internal __ieee754_acos/__ieee754_atan2 ifuncs that the exported wrappers tail-call)
ENTRIES = {
    "exp": 0x76470, "log": 0x76660, "atan": 0x76EE0, "acos": 0x77960,
    "atan2": 0x78060, "sin": 0x789B0, "cos": 0x791C0, "tan": 0x799D0,
}
NARGS = {"atan2": 2}
# the wrapper around __ieee754_* for these adds only errno handling (checked in the disassembly):
# exp/log/acos/atan2 wrappers (w_exp.c & co.) return the inner value unchanged for every input.

GPR64 = ["rax", "rbx", "rcx", "rdx", "rsi", "rdi", "rbp", "rsp"] + ["r%d" % i for i in range(8, 16)]
GPR = {}
for i, n in enumerate(["ax", "bx", "cx", "dx"]):
    GPR["r" + n] = (n, 64, 0); GPR["e" + n] = (n, 32, 0); GPR[n] = (n, 16, 0)
    GPR[n[0] + "l"] = (n, 8, 0); GPR[n[0] + "h"] = (n, 8, 8)
for n in ["si", "di", "bp", "sp"]:
    GPR["r" + n] = (n, 64, 0); GPR["e" + n] = (n, 32, 0); GPR[n] = (n, 16, 0); GPR[n + "l"] = (n, 8, 0)
for i in range(8, 16):
    GPR["r%d" % i] = ("r%d" % i, 64, 0); GPR["r%dd" % i] = ("r%d" % i, 32, 0)
    GPR["r%dw" % i] = ("r%d" % i, 16, 0); GPR["r%db" % i] = ("r%d" % i, 8, 0)
SIZES = {"QWORD": 64, "DWORD": 32, "WORD": 16, "BYTE": 8, "XMMWORD": 128}
MASK = {64: "0xFFFFFFFFFFFFFFFFull", 32: "0xFFFFFFFFull", 16: "0xFFFFull", 8: "0xFFull"}
CTYPE = {64: "uint64_t", 32: "uint32_t", 16: "uint16_t", 8: "uint8_t"}
STYPE = {64: "int64_t", 32: "int32_t", 16: "int16_t", 8: "int8_t"}


class Elf:
    def __init__(self, path):
        self.data = open(path, "rb").read()
        d = self.data
        phoff = struct.unpack_from("<Q", d, 0x20)[0]
        phentsize, phnum = struct.unpack_from("<HH", d, 0x36)
        self.segs = []
        for i in range(phnum):
            p_type, _f, off, va, _pa, filesz, _memsz, _al = struct.unpack_from("<IIQQQQQQ", d, phoff + i * phentsize)
            if p_type == 1:
                self.segs.append((va, off, filesz))

    def read(self, va, n):
        for v, o, s in self.segs:
            if v <= va and va + n <= v + s:
                return self.data[va - v + o: va - v + o + n]
        raise KeyError(hex(va))

    def q(self, va):
        return struct.unpack("<Q", self.read(va, 8))[0]


def disassemble(libm):
    out = subprocess.run(["objdump", "-d", "--no-show-raw-insn", "-M", "intel", libm],
                         check=True, capture_output=True, text=True).stdout
    ins = {}
    order = []
    for line in out.split("\n"):
        m = re.match(r"\s+([0-9a-f]+):\s+(.*)$", line)
        if not m:
            continue
        addr = int(m.group(1), 16)
        text = m.group(2).strip()
        comment = None
        if "#" in text:
            text, comment = text.split("#", 1)
            text = text.strip()
            comment = comment.strip()
        text = re.sub(r"\s*<[^>]*>", "", text)
        ins[addr] = (text, comment)
        order.append(addr)
    return ins, order


def split_ops(s):
    ops, depth, cur = [], 0, ""
    for ch in s:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip()); cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


class Fn:
    """Translate one function (entry address) into C."""

    def __init__(self, gen, name, entry, nargs, helper=False):
        self.g, self.name, self.entry, self.nargs, self.helper = gen, name, entry, nargs, helper
        self.lines = []
        self.labels = set()
        self.code = {}
        self.stack_used = False

    # ---- operands ----
    def rd_gpr(self, r):
        base, w, sh = GPR[r]
        v = "r_" + base
        if w == 64:
            return v
        if sh:
            return "((uint64_t)(uint8_t)(%s >> 8))" % v
        return "((uint64_t)(%s)%s)" % (CTYPE[w], v)

    def wr_gpr(self, r, expr):
        base, w, sh = GPR[r]
        v = "r_" + base
        if base == "sp":
            raise RuntimeError("rsp write")
        if w == 64:
            return "%s = (uint64_t)(%s);" % (v, expr)
        if w == 32:
            return "%s = (uint64_t)(uint32_t)(%s);" % (v, expr)
        if sh:
            return "%s = (%s & ~0xFF00ull) | ((uint64_t)(uint8_t)(%s) << 8);" % (v, v, expr)
        return "%s = (%s & ~%s) | (uint64_t)(%s)(%s);" % (v, v, MASK[w], CTYPE[w], expr)

    def mem(self, op, comment, addr, delta):
        """-> (kind, size, c-expr-of-address or static address)."""
        m = re.match(r"(?:(\w+) PTR )?(?:(fs):)?(.*)$", op)
        size = SIZES.get(m.group(1), 64) if m.group(1) else None
        seg, body = m.group(2), m.group(3)
        if seg == "fs":
            return ("fs", size, body)
        assert body.startswith("[") and body.endswith("]"), op
        e = body[1:-1]
        if e.startswith("rip"):
            assert comment, (hex(addr), op)
            return ("static", size, int(comment.split()[0], 16))
        terms = re.findall(r"[+-]?[^+-]+", e)
        base, parts, disp = None, [], 0
        for t in terms:
            sign = -1 if t.startswith("-") else 1
            t = t.lstrip("+-")
            if re.match(r"^0x[0-9a-f]+$|^\d+$", t):
                disp += sign * int(t, 0)
            elif "*" in t:
                r, s = t.split("*")
                parts.append("%s * %d" % (self.rd_gpr(r), int(s)))
            else:
                if t == "rsp":
                    base = "rsp"
                else:
                    parts.append(self.rd_gpr(t))
        if base == "rsp":
            assert not parts, op
            return ("stack", size, delta + disp)
        expr = " + ".join(parts) if parts else "0"
        if disp:
            expr = "(%s + (uint64_t)%dll)" % (expr, disp)
        return ("dyn", size, expr)

    def load(self, op, comment, addr, delta, width=None):
        """value of a register / memory / immediate operand as uint64 c-expr."""
        if op in GPR:
            return self.rd_gpr(op)
        if re.match(r"^xmm\d+$", op):
            return "x" + op[3:]
        if re.match(r"^-?0x[0-9a-f]+$|^-?\d+$", op):
            v = int(op, 0)
            return "0x%Xull" % (v & 0xFFFFFFFFFFFFFFFF)
        kind, size, a = self.mem(op, comment, addr, delta)
        size = width or size
        if kind == "static":
            try:
                v = self.g.elf.q(a)
            except KeyError:
                v = 0
            if a >= 0xE5D80:      # .data / GOT (errno TLS offset): value irrelevant
                v = 0
            if size == 32:
                v &= 0xFFFFFFFF
            self.g.static_reads.add(a)
            return "0x%016Xull" % v
        if kind == "fs":
            return "0ull"        # stack-protector canary / errno TLS base: irrelevant
        if kind == "stack":
            self.stack_used = True
            return "gl_stk_ld%d(stk, %d)" % (size if size != 128 else 64, a + 256)
        self.g.dyn_loads += 1
        if size == 32:
            return "((uint64_t)(uint32_t)GL_TAB(%s))" % a
        return "GL_TAB(%s)" % a

    def store(self, op, comment, addr, delta, expr):
        if op in GPR:
            return self.wr_gpr(op, expr)
        if re.match(r"^xmm\d+$", op):
            return "x%s = %s;" % (op[3:], expr)
        kind, size, a = self.mem(op, comment, addr, delta)
        if kind == "fs":
            return "/* errno */"
        if kind == "stack":
            self.stack_used = True
            return "gl_stk_st%d(stk, %d, %s);" % (size if size != 128 else 64, a + 256, expr)
        raise RuntimeError("store to %s at %x" % (op, addr))

    # ---- control flow ----
    def discover(self, ins):
        """Instructions reachable from the entry; stack delta per instruction."""
        starts = self.g.func_starts
        nxt = min([s for s in starts if s > self.entry] + [1 << 40])
        self.hi = nxt
        work = [(self.entry, 0)]
        seen = {}
        while work:
            a, d = work.pop()
            while True:
                if a in seen:
                    assert seen[a] == d, ("stack delta mismatch", hex(a))
                    break
                seen[a] = d
                text, comment = ins[a]
                mn = text.split()[0] if text else ""
                ops = split_ops(text[len(mn):]) if text else []
                self.code[a] = (text, comment, d)
                idx = self.g.order_idx[a]
                fall = self.g.order[idx + 1]
                if mn == "push":
                    d -= 8
                elif mn == "pop":
                    d += 8
                elif mn == "sub" and ops and ops[0] == "rsp":
                    d -= int(ops[1], 0)
                elif mn == "add" and ops and ops[0] == "rsp":
                    d += int(ops[1], 0)
                if mn == "ret":
                    break
                if mn == "jmp":
                    t = int(ops[0], 16)
                    if self.entry <= t < self.hi:
                        self.labels.add(t)
                        a = t
                        continue
                    self.g.need_helper(t)
                    break
                if mn.startswith("j"):
                    t = int(ops[0], 16)
                    if self.entry <= t < self.hi:
                        self.labels.add(t)
                        work.append((t, d))
                    else:
                        raise RuntimeError("conditional jump out of function at %x" % a)
                if mn == "call":
                    t = int(ops[0], 16)
                    name = self.g.call_name(t)
                    if name == "stack_chk_fail":
                        break
                a = fall

    # ---- translation ----
    def cond(self, cc):
        return {
            "a": "(!cf && !zf)", "nbe": "(!cf && !zf)", "ae": "(!cf)", "nb": "(!cf)", "nc": "(!cf)",
            "b": "(cf)", "c": "(cf)", "nae": "(cf)", "be": "(cf || zf)", "na": "(cf || zf)",
            "e": "(zf)", "z": "(zf)", "ne": "(!zf)", "nz": "(!zf)",
            "g": "(!zf && sf == of)", "nle": "(!zf && sf == of)", "ge": "(sf == of)", "nl": "(sf == of)",
            "l": "(sf != of)", "nge": "(sf != of)", "le": "(zf || sf != of)", "ng": "(zf || sf != of)",
            "s": "(sf)", "ns": "(!sf)", "p": "(pf)", "pe": "(pf)", "np": "(!pf)", "po": "(!pf)",
        }[cc]

    def width_of(self, op):
        if op in GPR:
            return GPR[op][1]
        m = re.match(r"(\w+) PTR", op)
        if m:
            return SIZES[m.group(1)]
        return None

    def int_flags(self, w, res, a=None, b=None, kind="logic"):
        """flag statements for an integer result of width w."""
        t = CTYPE[w]
        s = ["{ %s r_ = (%s)(%s);" % (t, t, res),
             "zf = (r_ == 0); sf = (int)(r_ >> %d); pf = !__builtin_parity((unsigned)(r_ & 0xFF));" % (w - 1)]
        if kind == "logic":
            s.append("cf = 0; of = 0;")
        elif kind == "sub":
            s.append("cf = ((%s)(%s) < (%s)(%s));" % (t, a, t, b))
            s.append("of = (int)((((%s)(%s) ^ (%s)(%s)) & ((%s)(%s) ^ r_)) >> %d);" % (t, a, t, b, t, a, w - 1))
        elif kind == "add":
            s.append("cf = (r_ < (%s)(%s));" % (t, a))
            s.append("of = (int)((((%s)(%s) ^ r_) & ((%s)(%s) ^ r_)) >> %d);" % (t, a, t, b, w - 1))
        s.append("}")
        return " ".join(s)

    def emit(self, a):
        text, comment, d = self.code[a]
        mn = text.split()[0] if text else "nop"
        ops = split_ops(text[len(mn):])
        L = lambda op, w=None: self.load(op, comment, a, d, w)
        S = lambda op, e: self.store(op, comment, a, d, e)
        out = []
        F = lambda e: "gl_f(%s)" % e
        U = lambda e: "gl_u(%s)" % e
        if ops and ops[0] == "rsp" and mn in ("add", "sub"):
            pass                                     # stack pointer: tracked statically (discover)
        elif mn in ("endbr64", "nop", "cs", "xchg", "vstmxcsr", "vldmxcsr") or mn.startswith("nop"):
            if mn == "xchg":
                assert ops == ["ax", "ax"], text
            if mn == "vstmxcsr":
                out.append(S(ops[0], "0x1F80ull"))   # default MXCSR: round to nearest, all masked
        elif mn in ("mov", "movabs", "vmovq", "movq", "movd", "vmovd"):
            w = self.width_of(ops[0]) or self.width_of(ops[1]) or 64
            v = L(ops[1], w if not re.match(r"^xmm", ops[1]) else None)
            out.append(S(ops[0], v))
        elif mn in ("vmovsd", "movsd", "movapd", "vmovapd", "movaps", "vmovaps"):
            if len(ops) == 3:
                out.append(S(ops[0], L(ops[2])))
            else:
                out.append(S(ops[0], L(ops[1], 64)))
        elif mn == "movsxd":
            out.append(S(ops[0], "(uint64_t)(int64_t)(int32_t)(%s)" % L(ops[1], 32)))
        elif mn == "cdqe":
            out.append("r_ax = (uint64_t)(int64_t)(int32_t)r_ax;")
        elif mn == "lea":
            kind, size, e = self.mem(ops[1], comment, a, d)
            if kind == "static":
                out.append(S(ops[0], "0x%Xull" % e))
                self.g.lea_bases.add(e)
            elif kind == "stack":
                out.append(S(ops[0], "0ull /* stack address: only passed to __branred */"))
            else:
                assert kind == "dyn", text
                out.append(S(ops[0], e))
        elif mn in ("add", "sub", "and", "or", "xor", "cmp", "test"):
            w = self.width_of(ops[0])
            x, y = L(ops[0], w), L(ops[1], w)
            if mn == "xor" and ops[0] == ops[1]:
                y = x
            t = CTYPE[w]
            res = {"add": "(%s)+(%s)", "sub": "(%s)-(%s)", "cmp": "(%s)-(%s)", "and": "(%s)&(%s)",
                   "test": "(%s)&(%s)", "or": "(%s)|(%s)", "xor": "(%s)^(%s)"}[mn] % (x, y)
            kind = {"add": "add", "sub": "sub", "cmp": "sub"}.get(mn, "logic")
            out.append(self.int_flags(w, res, x, y, kind))
            if mn not in ("cmp", "test"):
                out.append(S(ops[0], "(%s)(%s)" % (t, res)))
        elif mn in ("shl", "shr", "sar"):
            w = self.width_of(ops[0])
            x = L(ops[0], w)
            n = int(ops[1], 0) if len(ops) > 1 else 1
            t = CTYPE[w]
            if mn == "shl":
                res = "(%s)((%s)(%s) << %d)" % (t, t, x, n)
            elif mn == "shr":
                res = "(%s)((%s)(%s) >> %d)" % (t, t, x, n)
            else:
                res = "(%s)((%s)(%s) >> %d)" % (t, STYPE[w], x, n)
            out.append(self.int_flags(w, res))     # cf/of of shifts are never consumed here
            out.append(S(ops[0], res))
        elif mn == "imul":
            w = self.width_of(ops[0])
            t = CTYPE[w]
            if len(ops) == 3:
                res = "(%s)((%s)(%s) * (%s)(%s))" % (t, t, L(ops[1], w), t, L(ops[2], w))
            else:
                res = "(%s)((%s)(%s) * (%s)(%s))" % (t, t, L(ops[0], w), t, L(ops[1], w))
            out.append(S(ops[0], res))
        elif mn.startswith("cmov"):
            w = self.width_of(ops[0])
            out.append("if %s { %s }" % (self.cond(mn[4:]), S(ops[0], L(ops[1], w))))
            if w == 32:   # a 32-bit cmov zero-extends its destination even when not taken
                out.append("else { %s }" % S(ops[0], L(ops[0], 32)))
        elif mn.startswith("set"):
            out.append(S(ops[0], "(uint64_t)%s" % self.cond(mn[3:])))
        elif mn in ("push",):
            self.stack_used = True
            out.append("gl_stk_st64(stk, %d, %s);" % (d - 8 + 256, L(ops[0])))
        elif mn in ("pop",):
            self.stack_used = True
            out.append(S(ops[0], "gl_stk_ld64(stk, %d)" % (d + 256)))
        elif mn in ("vaddsd", "vsubsd", "vmulsd", "vdivsd", "addsd", "subsd", "mulsd", "divsd"):
            opc = {"add": "+", "sub": "-", "mul": "*", "div": "/"}[mn.lstrip("v")[:3]]
            if mn.startswith("v"):
                x, y = L(ops[1]), L(ops[2], 64)
            else:
                x, y = L(ops[0]), L(ops[1], 64)
            out.append(S(ops[0], U("%s %s %s" % (F(x), opc, F(y)))))
        elif mn in ("vandpd", "vorpd", "vxorpd", "vxorps", "vandnpd", "andpd", "orpd", "xorpd", "xorps", "andnpd"):
            if mn.startswith("v"):
                x, y = L(ops[1]), L(ops[2], 64)
            else:
                x, y = L(ops[0]), L(ops[1], 64)
            base = mn.lstrip("v")[:-2]
            if base == "xor" and x == y:
                out.append(S(ops[0], "0ull"))
            else:
                e = {"and": "(%s) & (%s)", "or": "(%s) | (%s)", "xor": "(%s) ^ (%s)", "andn": "~(%s) & (%s)"}[base] % (x, y)
                out.append(S(ops[0], e))
        elif re.match(r"v?fn?m(add|sub)(132|213|231)sd", mn):
            m = re.match(r"v?f(n?)m(add|sub)(132|213|231)sd", mn)
            neg, kind, form = m.group(1) == "n", m.group(2), m.group(3)
            a1, a2, a3 = L(ops[0]), L(ops[1]), L(ops[2], 64)
            p, q, c = {"132": (a1, a3, a2), "213": (a2, a1, a3), "231": (a2, a3, a1)}[form]
            pe = ("-" if neg else "") + F(p)
            ce = ("-" if kind == "sub" else "") + F(c)
            out.append(S(ops[0], U("gl_fma(%s, %s, %s)" % (pe, F(q), ce))))
        elif mn in ("vcomisd", "vucomisd", "comisd", "ucomisd"):
            x, y = L(ops[0]), L(ops[1], 64)
            out.append("{ double a_ = %s, b_ = %s; int u_ = (a_ != a_) || (b_ != b_);" % (F(x), F(y)))
            out.append("zf = u_ || (a_ == b_); pf = u_; cf = u_ || (a_ < b_); sf = 0; of = 0; }")
        elif mn in ("vcmpltsd", "vcmpnltsd", "vcmpnlesd", "vcmplesd", "vcmpeqsd", "vcmpneqsd"):
            x, y = L(ops[1]), L(ops[2], 64)
            c = {"vcmpltsd": "(a_ < b_)", "vcmpnltsd": "!(a_ < b_)", "vcmpnlesd": "!(a_ <= b_)",
                 "vcmplesd": "(a_ <= b_)", "vcmpeqsd": "(a_ == b_)", "vcmpneqsd": "!(a_ == b_)"}[mn]
            out.append("{ double a_ = %s, b_ = %s; %s }" % (F(x), F(y), S(ops[0], "(%s ? ~0ull : 0ull)" % c)))
        elif mn == "vblendvpd":
            x, y, m_ = L(ops[1]), L(ops[2], 64), L(ops[3])
            out.append(S(ops[0], "((int64_t)(%s) < 0 ? (%s) : (%s))" % (m_, y, x)))
        elif mn in ("vcvttsd2si", "cvttsd2si"):
            w = self.width_of(ops[0])
            out.append(S(ops[0], "gl_cvtt%d(%s)" % (w, F(L(ops[1], 64)))))
        elif mn in ("vcvtsi2sd", "cvtsi2sd"):
            src = ops[2] if mn.startswith("v") else ops[1]
            w = self.width_of(src)
            out.append(S(ops[0], U("(double)(%s)(%s)" % (STYPE[w], L(src, w)))))
        elif mn == "ret":
            out.append("return x0;")
        elif mn == "jmp":
            t = int(ops[0], 16)
            if self.entry <= t < self.hi:
                out.append("goto L_%x;" % t)
            else:
                out.append("return gl_h_%x(r_di, x0, x1);" % t)
        elif mn.startswith("j"):
            t = int(ops[0], 16)
            out.append("if %s goto L_%x;" % (self.cond(mn[1:]), t))
        elif mn == "call":
            t = int(ops[0], 16)
            name = self.g.call_name(t)
            if name == "stack_chk_fail":
                out.append("return x0; /* stack protector: unreachable */")
            else:
                # __branred: |x| >= 105414350 -- outside the tracer's domain
                out.append("return 0x7FF8000000000000ull; /* huge-argument reduction (%s) not translated */" % name)
        else:
            raise RuntimeError("unhandled %x: %s" % (a, text))
        return out

    def translate(self, ins):
        self.discover(ins)
        addrs = sorted(self.code)
        out = []
        for i, a in enumerate(addrs):
            if a in self.labels or a == self.entry:
                out.append("L_%x:;" % a)
            text = self.code[a][0]
            st = self.emit(a)
            out.append("    " + " ".join(st) + "   /* %x: %s */" % (a, text.replace("*/", "* /")))
            mn = text.split()[0] if text else ""
            nxt = self.g.order[self.g.order_idx[a] + 1]
            if mn not in ("ret", "jmp", "call") and not (i + 1 < len(addrs) and addrs[i + 1] == nxt):
                raise RuntimeError("fallthrough of %x not translated" % a)
        return out


class Gen:
    def __init__(self, libm):
        self.elf = Elf(libm)
        self.ins, self.order = disassemble(libm)
        self.order_idx = {a: i for i, a in enumerate(self.order)}
        self.func_starts = sorted(a for a, (t, c) in self.ins.items() if t == "endbr64")
        self.helpers = {}
        self.pending = []
        self.static_reads = set()
        self.lea_bases = set()
        self.dyn_loads = 0
        plt = {}
        self.plt = plt

    def call_name(self, t):
        text, comment = self.ins.get(t, ("", None))
        if t == 0xE240:
            return "stack_chk_fail"
        return "fn_%x" % t

    def need_helper(self, t):
        if t not in self.helpers and t not in self.pending:
            self.pending.append(t)


def build_id(libm):
    out = subprocess.run(["readelf", "-n", libm], capture_output=True, text=True).stdout
    m = re.search(r"Build ID: ([0-9a-f]+)", out)
    return m.group(1) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libm", default="/lib/x86_64-linux-gnu/libm.so.6")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..",
                                                  "minimal_volumetric_path_tracer_amd", "csrc", "vpt_glibc.h"))
    args = ap.parse_args()
    bid = build_id(args.libm)
    if bid != BUILD_ID:
        sys.exit("libm build-id %s != pinned %s: re-derive ENTRIES for this library" % (bid, BUILD_ID))
    g = Gen(args.libm)
    fns = []
    for name, entry in ENTRIES.items():
        f = Fn(g, name, entry, NARGS.get(name, 1))
        fns.append((f, f.translate(g.ins)))
    helpers = []
    while g.pending:
        t = g.pending.pop()
        f = Fn(g, "h_%x" % t, t, 2, helper=True)
        g.helpers[t] = f
        helpers.append((f, f.translate(g.ins)))
    # table extract: from the lowest dynamic base to the end of the last table (bounded by the
    # next non-table object: we take every base's region up to the following base, and the last
    # base's up to its known extent)
    lo = min(g.lea_bases)
    hi = TABLE_END
    blob = g.elf.read(lo, hi - lo)
    words = struct.unpack("<%dQ" % ((hi - lo) // 8), blob)
    with open(args.out, "w") as fh:
        w = fh.write
        w("/* GENERATED by scripts/gen_glibc_libm.py from libm.so.6 build-id %s (Ubuntu GLIBC\n" % BUILD_ID)
        w(" * 2.35-0ubuntu3.12), x86-64 FMA variants.  Do not edit.  GNU C Library, LGPL-2.1-or-later\n")
        w(" * (LICENSE-glibc-derived.md: the notice and how libvpt.so is rebuilt from these sources).\n")
        w(" *\n * gl_exp, gl_log, gl_sin, gl_cos, gl_tan, gl_atan, gl_acos, gl_atan2: the same bits as the\n")
        w(" * reference's libm calls for every argument the tracer passes (tests/test_glibc_libm.py).\n")
        w(" * Register variables r_* (integer) and x* (low lane of xmm*, as bits); flags zf/cf/sf/of/pf.\n */\n")
        w("#ifndef VPT_GLIBC_H\n#define VPT_GLIBC_H\n#include \"vpt_glibc_rt.h\"\n\n")
        w("#if defined(__clang__)\n#pragma clang diagnostic push\n#pragma clang diagnostic ignored \"-Wunused-label\"\n")
        w("#pragma clang diagnostic ignored \"-Wunused-variable\"\n#pragma clang diagnostic ignored \"-Wunused-but-set-variable\"\n")
        w("#elif defined(__GNUC__)\n#pragma GCC diagnostic push\n#pragma GCC diagnostic ignored \"-Wunused-label\"\n")
        w("#pragma GCC diagnostic ignored \"-Wunused-variable\"\n#pragma GCC diagnostic ignored \"-Wunused-but-set-variable\"\n#endif\n\n")
        w("#define GL_TAB_LO 0x%Xull\n#define GL_TAB_WORDS %d\n" % (lo, len(words)))
        w("GL_TABLE_DECL(gl_tab, GL_TAB_WORDS) = {\n")
        for i in range(0, len(words), 4):
            w("    " + ", ".join("0x%016Xull" % x for x in words[i:i + 4]) + ",\n")
        w("};\n")
        w("#ifdef GL_CHECK_BOUNDS\nstatic uint64_t gl_tab_ld_checked(uint64_t a)\n{\n")
        w("    if (a < GL_TAB_LO || a >= GL_TAB_LO + 8ull * GL_TAB_WORDS || (a & 7)) {\n")
        w("        fprintf(stderr, \"gl_tab: address 0x%llx outside the table extract\\n\", (unsigned long long)a);\n")
        w("        abort();\n    }\n    return gl_tab[(a - GL_TAB_LO) >> 3];\n}\n#endif\n\n")
        for f, body in helpers:
            w("GL_FN uint64_t gl_h_%x(uint64_t r_di_in, uint64_t x0_in, uint64_t x1_in);\n" % f.entry)
        w("\n")
        for f, body in helpers:
            w("GL_FN uint64_t gl_h_%x(uint64_t r_di_in, uint64_t x0_in, uint64_t x1_in)\n{\n" % f.entry)
            w(prologue(f, "    r_di = r_di_in; x0 = x0_in; x1 = x1_in;\n", body))
            w("\n".join(body) + "\n}\n\n")
        for f, body in fns:
            args_ = "double a0" + (", double a1" if f.nargs == 2 else "")
            init = "    x0 = gl_u(a0);" + (" x1 = gl_u(a1);" if f.nargs == 2 else "") + "\n"
            w("GL_ENTRY double gl_%s(%s)\n{\n" % (f.name, args_))
            w(prologue(f, init, body))
            w("\n".join(body).replace("return x0;", "return gl_f(x0);").replace(
                "return gl_h_", "return gl_f(gl_h_").replace("(r_di, x0, x1);", "(r_di, x0, x1));").replace(
                "return 0x7FF8000000000000ull;", "return gl_f(0x7FF8000000000000ull);") + "\n}\n\n")
        w("#if defined(__clang__)\n#pragma clang diagnostic pop\n#elif defined(__GNUC__)\n#pragma GCC diagnostic pop\n#endif\n")
        w("#endif\n")
    print("wrote %s: %d functions, %d helpers, table %d words (0x%x..0x%x), %d dynamic loads" % (
        args.out, len(fns), len(helpers), len(words), lo, hi, g.dyn_loads))


def prologue(f, init, body):
    """declare only the registers the body (or the argument set-up) touches"""
    text = "\n".join(body) + init
    used = [r for r in GPR64 if r != "rsp" and re.search(r"\br_%s\b" % GPR[r][0], text)]
    if "r_di" not in [("r_" + GPR[r][0]) for r in used] and ("r_di" in text):
        used.append("rdi")
    regs = ("    uint64_t " + ", ".join("r_" + GPR[r][0] + " = 0" for r in used) + ";\n") if used else ""
    xs = [i for i in range(16) if re.search(r"\bx%d\b" % i, text)]
    xm = ("    uint64_t " + ", ".join("x%d = 0" % i for i in xs) + ";\n") if xs else ""
    fl = "    int zf = 0, cf = 0, sf = 0, of = 0, pf = 0;\n"
    st = "    unsigned char stk[320];\n" if f.stack_used else ""
    unused = "    (void)zf; (void)cf; (void)sf; (void)of; (void)pf;\n"
    return regs + xm + fl + st + unused + init


TABLE_END = 0xC2D80

if __name__ == "__main__":
    main()
