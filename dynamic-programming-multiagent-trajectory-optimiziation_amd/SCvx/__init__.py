"""Drop-in compatibility surface of the reference package `SCvx` (same module paths), backed by the
MI355X-native batched kernels of `scvx_hip`.  Put the directory containing this package on
sys.path instead of the reference root and `from SCvx.discretization.first_order_hold import
FirstOrderHold` resolves here."""
