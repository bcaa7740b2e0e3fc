"""Hand-offs between backward passes, keyed on the gradient tensor itself.

A backward that produces a gradient tensor can compute something its
consumer's backward would otherwise compute from that tensor in a pass of its
own (the loss kernel sums dz's columns and writes dz / deg as it stores dz;
the input-gradient kernel applies the ReLU mask and sums dx's columns). The
value is attached to the consuming autograd node as a ``GradHandoff`` and
taken only if the gradient that node receives is *the same tensor object*,
unmodified since:

* identity is a weak reference to the tensor, not its address: a freed
  gradient whose storage the caching allocator hands to a later tensor can
  never match (the reference is dead, and the value is dropped with it);
* the version counter rules out in-place updates in between (a gradient
  summed in place with another consumer's, a user's ``mul_``);
* everything handed over is a function of the tensor's contents alone, so a
  match is correct whenever and however often it is taken.

Anything else (autograd summed two consumers' gradients into a new tensor,
``autograd.grad`` stopped at the tensor and the caller passed another one) is
a miss, and the consumer computes the value itself.
"""
import weakref

__all__ = ["GradHandoff", "take", "output_ref", "is_output", "stats"]

# hand-offs taken / offered but missed, since import (tests and studies read it)
stats = {"taken": 0, "missed": 0}


class GradHandoff(object):
    """``value`` computed from ``grad``, valid for that tensor object at its
    current version; dropped as soon as the tensor is freed."""

    __slots__ = ("_ref", "_version", "_holder")

    def __init__(self, grad, value):
        holder = [value]
        self._holder = holder
        self._version = grad._version
        # the callback holds the list, not self: no cycle keeps the value alive
        self._ref = weakref.ref(grad, lambda _r, h=holder: h.clear())

    def take(self, grad):
        """The value if ``grad`` is the tensor it was computed from, unmodified."""
        if self._holder and self._ref() is grad and grad._version == self._version:
            stats["taken"] += 1
            return self._holder[0]
        stats["missed"] += 1
        return None


def take(handoff, grad):
    """``handoff.take(grad)``, None for no hand-off."""
    return None if handoff is None else handoff.take(grad)


def output_ref(out):
    """A weak reference to an autograd Function's output, stored on its node."""
    return weakref.ref(out)


def is_output(node, t):
    """Is ``t`` the very tensor ``node`` returned (not a view, not a copy)?"""
    ref = getattr(node, "out_ref", None)
    return ref is not None and ref() is t
