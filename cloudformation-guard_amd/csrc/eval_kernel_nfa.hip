// The evaluator kernels with the regex NFA simulation compiled in (eval_core.inc nfa_run): launched
// instead of eval_kernel.hip's for a session whose rules hold a regex with no DFA within the compile
// limits (regex_dfa.cpp nfa_fallback).  Same source, GG_NFA 1: kernel names suffixed _nfa.
#define GG_NFA 1
#include "eval_kernel.hip"
