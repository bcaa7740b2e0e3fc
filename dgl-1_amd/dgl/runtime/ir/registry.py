"""Opcode table: name, argument and result types, executor class of every IR
operation (counterpart of python/dgl/runtime/ir/registry.py; filled in by
executor.py)."""
from __future__ import absolute_import

__all__ = ["IR_REGISTRY", "op_name"]

IR_REGISTRY = {}


def op_name(opcode):
    return IR_REGISTRY[opcode]["name"]
