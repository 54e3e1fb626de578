"""Per-call latency of the drop-in module on short and long pairs (what an unchanged caller such
as IRMethods.wf_score or the GUI pays per wagnerFisher / create_paths / generate_es call)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd")]
os.chdir(os.path.join(REPO, "tests", "golden"))
import StringEditDistance as SED  # noqa: E402
import synth  # noqa: E402

def per_call(f, k):
    f()
    t0 = time.perf_counter()
    for _ in range(k):
        f()
    return (time.perf_counter() - t0) / k * 1e3

a, b = "AAAAAAAAAAAGGGAGCGAAGUCAAGGCCC", "AAAAAAAAAAAGUGCUACGACAUUUGGGGGU"
s1, s2 = synth.pair_strings(0, 4096, 4096)
print("wf_score-style distance, 30 nt pair: %.3f ms/call" % per_call(lambda: SED.wagnerFisher(a, b)[-1][-1].value, 300))
print("distance + canonical ES, 30 nt pair: %.3f ms/call" %
      per_call(lambda: SED.generate_es(SED.create_paths(SED.wagnerFisher(a, b))[0], a, b), 300))
print("distance, 4096^2 pair (user costs): %.3f ms/call" % per_call(lambda: SED.wagnerFisher(s1, s2, True)[-1][-1].value, 20))
print("distance + canonical ES, 4096^2 pair: %.3f ms/call" %
      per_call(lambda: SED.generate_es(SED.create_paths(SED.wagnerFisher(s1, s2, True))[0], s1, s2), 20))
print("ES + patching round trip, 4096^2 pair: %.3f ms/call" %
      per_call(lambda: SED.patching(SED.generate_es(SED.create_paths(SED.wagnerFisher(s1, s2, True))[0], s1, s2), s1), 20))
