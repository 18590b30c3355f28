# dev: the zeroing stream's block-row chain waits for the look-ahead (a) instead of the panel
import sys
p = sys.argv[1] + '/math_amd/csrc/cholesky.hip'
s = open(p).read()
old = '''    if (zero_parts && J / NB2 < rows_prog) {  // this panel is final: its block row's inverses may start
      if (!(pe_ev[J / NB2] = smg_event(ctx, nev++))) return SMG_ERR_HIP;
      SMG_HIP_TRY(hipEventRecord(pe_ev[J / NB2], ctx->stream));
    }
'''
assert old in s
s = s.replace(old, '')
old = '''    SMG_HIP_TRY(hipEventRecord(E, ctx->stream));
    F = nullptr;'''
new = '''    SMG_HIP_TRY(hipEventRecord(E, ctx->stream));
    // this panel's block row starts on the zeroing stream once the look-ahead (a) is done:
    // (a) has the gap to itself
    if (zero_parts && J / NB2 < rows_prog) pe_ev[J / NB2] = E;
    F = nullptr;'''
assert old in s
s = s.replace(old, new)
open(p, 'w').write(s)
