"""cilium_amd — MI355X-native batched L7 policy evaluator for Cilium's L7 rule
model (PortRuleHTTP / PortRuleKafka).  The product is libl7match.so (C ABI,
include/l7match.h); `cilium_amd.l7match` is its Python binding."""
__all__ = ["l7match"]
