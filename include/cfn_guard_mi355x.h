/* C ABI of the MI355X batch evaluator for AWS CloudFormation Guard rules.
 *
 * Drop-in for guard-ffi (reference: guard-ffi/src/lib.rs:32-47, guard-ffi/src/types.rs:4-8,
 * guard-ffi/example/cfn_guard.h): same struct layouts, same error codes
 * (guard-ffi/src/errors.rs:12-38), same JSON bytes.
 * All entry points evaluate on the GPU; without a HIP device they fail with code -1.
 * Devices: the single-device entry points use the process default device -- the HIP device current on
 * the thread of the first call (a one-process-per-GPU job sets it per rank, e.g.
 * torch.cuda.set_device(LOCAL_RANK)), or GG_DEVICE=<ordinal>.  The *_devices / *_gpus entry points take
 * a device list and shard the documents over it inside the library (one host thread per device); a
 * session (gg_session_*) is bound to the device current when it first uploads.  Calls may come from any
 * host thread, concurrently.
 */
#ifndef CFN_GUARD_MI355X_H
#define CFN_GUARD_MI355X_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* guard-ffi/example/cfn_guard.h: extern_err_t (ffi-support ExternError) */
typedef struct {
  int32_t code;
  char *message;
} extern_err_t;

/* guard-ffi/example/cfn_guard.h / src/types.rs:4-8 FfiValidateInput */
typedef struct {
  const char *content;
  const char *file_name;
} validate_input_t;

/* Replaces guard-ffi `cfn_guard_run_checks` (guard-ffi/src/lib.rs:32-45 -> run_checks,
 * guard/src/commands/helper.rs:25-87): one document x one rules file, pretty FileReport JSON;
 * verbose == true: the pretty serde EventRecord tree of the evaluation (helper.rs:62-64). */
char *cfn_guard_run_checks(validate_input_t data, validate_input_t rules, bool verbose, extern_err_t *err);

/* Replaces guard-ffi `cfn_guard_free_string` (guard-ffi/src/lib.rs:47). NULL is a no-op. */
void cfn_guard_free_string(char *s);

/* Batched `cfn-guard validate --structured -o json -S none` (guard/src/commands/validate.rs:391-403,
 * commands/reporters/validate/structured.rs:99-133): n_docs documents x n_rules rules files.
 * *exit_code receives 0 / 19 / 5 / -1 like the CLI (commands/mod.rs:69-73, main.rs:35-42). */
char *cfn_guard_validate_batch(const validate_input_t *docs, size_t n_docs, const validate_input_t *rules,
                               size_t n_rules, int32_t *exit_code, extern_err_t *err);

/* Output formats of `validate --structured -o <format>` (commands/validate.rs:143-200,
 * reporters/validate/structured.rs:124-133, sarif.rs, xml.rs). */
#define CFN_GUARD_OUTPUT_JSON 0
#define CFN_GUARD_OUTPUT_YAML 1
#define CFN_GUARD_OUTPUT_SARIF 2
#define CFN_GUARD_OUTPUT_JUNIT 3
/* cfn_guard_validate_batch with `-o json|yaml|sarif|junit` (byte-identical to the CLI's output). */
char *cfn_guard_validate_batch_format(const validate_input_t *docs, size_t n_docs, const validate_input_t *rules,
                                      size_t n_rules, int32_t output_format, int32_t *exit_code, extern_err_t *err);

/* cfn_guard_validate_batch_format with input parameters: `validate --structured -i <params>...`
 * (commands/validate.rs:317-350; reporters/validate/structured.rs:51-65).  params: the parameter
 * files in the order the CLI walks its -i arguments (files and sorted directory listings); they are
 * merged in that order with PathAwareValue::merge (path_value.rs:889-919) and the result is merged
 * into every data file.  A conflict between parameter files is the reference's MultipleValues (9) /
 * IncompatibleError (11) abort; between the parameters and a data file the reference unwraps the
 * merge and panics: code -1, message "called `Result::unwrap()` on an `Err` value: ...". */
char *cfn_guard_validate_batch_params(const validate_input_t *docs, size_t n_docs, const validate_input_t *rules,
                                      size_t n_rules, const validate_input_t *params, size_t n_params,
                                      int32_t output_format, int32_t *exit_code, extern_err_t *err);

/* cfn_guard_validate_batch_params over several GPUs of this process (SURVEY.md 8(b) "n_gpus", 8(e)): the
 * documents are split into contiguous ranges balanced by text bytes, one per entry of `devices` (HIP
 * ordinals; an ordinal may repeat -- two shards on one GPU), each range loaded, evaluated and fetched on its
 * own host thread and device, and the shards' reports joined in document order on the host: the same bytes
 * and exit code as the one-device call, with its error precedence.  devices NULL: every visible device
 * (n_devices ignored).  Replaces, for a caller that owns the node's GPUs in one process, the per-file loop
 * of CommonStructuredReporter::report (reporters/validate/structured.rs:99-133). */
char *cfn_guard_validate_batch_devices(const validate_input_t *docs, size_t n_docs, const validate_input_t *rules,
                                       size_t n_rules, const validate_input_t *params, size_t n_params,
                                       int32_t output_format, const int32_t *devices, size_t n_devices,
                                       int32_t *exit_code, extern_err_t *err);
/* cfn_guard_validate_batch_format(JSON) streamed for batches whose report does not fit one string: the
 * documents run in chunks of chunk_docs (0: 262144) on two alternating sessions (the next chunk loads and
 * evaluates while this one's report renders on the device), and the report's bytes go to write(ctx, data,
 * len) in order (a nonzero return aborts).  Returns 0 with *exit_code as the one-string call's, or -1 with
 * err on an abort -- after the chunks before the failing one were written (the caller drops that prefix).
 * Threads: `write` is called from the calling thread or from threads the library owns (a chunk's report
 * thread or its copy thread), never two calls at once, always in document order, and never after this
 * function has returned. */
typedef int32_t (*cfn_guard_write_fn)(void *ctx, const char *data, size_t len);
int32_t cfn_guard_validate_batch_stream(const validate_input_t *docs, size_t n_docs, const validate_input_t *rules,
                                        size_t n_rules, size_t chunk_docs, cfn_guard_write_fn write, void *ctx,
                                        int32_t *exit_code, extern_err_t *err);
/* The same stream over several GPUs of the process: chunk k (chunk_docs documents, 0 = 16384) is loaded,
 * evaluated and rendered on devices[k % n_devices] (NULL: every visible device; ordinals may repeat), each
 * device's pipeline on a host thread of its own; the reports reach `write` in document order from the
 * calling thread.  Host memory holds at most two chunks' reports per device.  One device: exactly
 * cfn_guard_validate_batch_stream on that device.  Same bytes, exit code and error behaviour. */
int32_t cfn_guard_validate_batch_stream_devices(const validate_input_t *docs, size_t n_docs,
                                                const validate_input_t *rules, size_t n_rules, size_t chunk_docs,
                                                const int32_t *devices, size_t n_devices, cfn_guard_write_fn write,
                                                void *ctx, int32_t *exit_code, extern_err_t *err);
/* The streamed entries with the one-string call's whole structured contract (cfn_guard_validate_batch_params /
 * _devices: `validate --structured -o json|yaml|sarif|junit [-i <params>]*`, structured.rs:99-133,
 * validate.rs:317-350): output_format CFN_GUARD_OUTPUT_* (JSON, YAML, SARIF, JUNIT), params merged into every
 * data file, chunks of chunk_docs documents (0: 262144 on one device, 16384 per chunk over several) on
 * devices[k % n_devices] (NULL: the process default device).  The bytes `write` receives are the one-string
 * call's, in document order.  JSON and YAML write each chunk while later ones run (two chunks' reports per
 * device in host memory); SARIF and JUnit put their frame -- the FAILed documents' artifacts, the test totals --
 * before every result, so they keep every chunk's evaluated results on its device until the last chunk is
 * evaluated (about 20 GB of HBM per million CloudFormation templates, no report text), then write.  Errors follow
 * the one-string call's precedence; JSON / YAML may have written the chunks before the failing one (a prefix to
 * drop), SARIF / JUnit write nothing before an error.  JSON without params is cfn_guard_validate_batch_stream
 * (one device) / _stream_devices. */
int32_t cfn_guard_validate_batch_stream_ex(const validate_input_t *docs, size_t n_docs, const validate_input_t *rules,
                                           size_t n_rules, const validate_input_t *params, size_t n_params,
                                           int32_t output_format, size_t chunk_docs, const int32_t *devices,
                                           size_t n_devices, cfn_guard_write_fn write, void *ctx, int32_t *exit_code,
                                           extern_err_t *err);
/* synthetic corpora as validate inputs (bench.py): format 0 JSON (synth.cfn_doc), 1 block-style YAML */
typedef struct gg_texts gg_texts;
gg_texts *gg_synth_texts(uint64_t first, size_t n, int32_t n_resources, int32_t format, int32_t nthreads);
const validate_input_t *gg_texts_inputs(gg_texts *t);
void gg_texts_free(gg_texts *t);
/* the n_gpus form of SURVEY.md 8(b): devices 0 .. n_gpus - 1 (n_gpus <= 0: every visible device), no -i. */
char *cfn_guard_validate_batch_gpus(const validate_input_t *docs, size_t n_docs, const validate_input_t *rules,
                                    size_t n_rules, int32_t output_format, int32_t n_gpus, int32_t *exit_code,
                                    extern_err_t *err);

/* `cfn-guard validate [-r <rules>]+ [-d <data>]+ [-i <params>]* [-o single-line-summary|json|yaml]
 * [-S <summary>] [--verbose] [--print-json]` -- the console reporters, not --structured
 * (commands/validate.rs:253-487, 552-596, 690-758; reporters/validate/{summary_table,cfn,tf,
 * generic_summary,common}.rs).  rules and docs in the CLI's walk order (file name = what the CLI
 * prints for it); show_summary: CFN_GUARD_SUMMARY_* bits (the CLI default is _FAIL; 0 = `-S none`);
 * output_format: CFN_GUARD_OUTPUT_TEXT (single-line-summary), _JSON or _YAML; flags:
 * CFN_GUARD_CONSOLE_VERBOSE | CFN_GUARD_CONSOLE_PRINT_JSON.  Returns stdout (free with
 * cfn_guard_free_string); *err_text gets stderr (rules-file parse errors, "Error occurred ..."), or NULL.
 * *exit_code: 0 / 19 (a rule FAILed) / 5 (a rules file did not parse; the last non-zero code wins) /
 * -1 with err set when evaluation aborted -- stdout then holds what was written before the abort. */
#define CFN_GUARD_SUMMARY_PASS 1u
#define CFN_GUARD_SUMMARY_FAIL 2u
#define CFN_GUARD_SUMMARY_SKIP 4u
#define CFN_GUARD_CONSOLE_VERBOSE 1u
#define CFN_GUARD_CONSOLE_PRINT_JSON 2u
char *cfn_guard_validate_console(const validate_input_t *docs, size_t n_docs, const validate_input_t *rules,
                                 size_t n_rules, const validate_input_t *params, size_t n_params, uint32_t show_summary,
                                 int32_t output_format, uint32_t flags, int32_t *exit_code, char **err_text,
                                 extern_err_t *err);

/* `cfn-guard test -r <rules> -t <spec files> [-o json|yaml|junit]` (commands/test.rs,
 * reporters/test/generic.rs and structured.rs): one rules file x n_specs test-spec files
 * (YAML / JSON `Vec<TestSpec>`); output_format CFN_GUARD_OUTPUT_TEXT (the default text report),
 * _JSON, _YAML or _JUNIT.  *exit_code: 0 / 7 (a test failed) / 1 (a spec file did not parse). */
#define CFN_GUARD_OUTPUT_TEXT 4
char *cfn_guard_test(validate_input_t rules, const validate_input_t *specs, size_t n_specs, int32_t output_format,
                     int32_t *exit_code, extern_err_t *err);
/* cfn_guard_test with `--verbose` (text only): each test case's EventRecord tree printed as
 * print_verbose_tree does (commands/validate.rs:666-687, reporters/test/generic.rs:116-118); verbose
 * with a structured format is the reference's IllegalArguments (18, test.rs:134-137). */
char *cfn_guard_test_ex(validate_input_t rules, const validate_input_t *specs, size_t n_specs, int32_t output_format,
                        bool verbose, int32_t *exit_code, extern_err_t *err);

/* `cfn-guard test -d <dir> [-o json|yaml|junit]` (commands/test.rs:143-165): n_rules rules files, rules
 * file i with the spec_counts[i] test-spec files that follow each other in `specs` (the directory's
 * pairing of a rules file with its tests, done by the caller as OrderedTestDirectory does).  Text:
 * "Testing Guard File ..." sections (test.rs:221-283); json / yaml / junit: one Vec<TestResult>
 * (test.rs:383-456); verbose (text only) as cfn_guard_test_ex.  *exit_code as cfn_guard_test, folded
 * over the rules files. */
char *cfn_guard_test_dir(const validate_input_t *rules, size_t n_rules, const validate_input_t *specs,
                         const size_t *spec_counts, int32_t output_format, bool verbose, int32_t *exit_code,
                         extern_err_t *err);

/* ---- session API (documents resident in HBM across evaluations; used by bench.py/tests) ---- */
typedef struct gg_session gg_session;
gg_session *gg_session_new(void);
void gg_session_free(gg_session *s);
int32_t gg_session_add_rules(gg_session *s, const char *text, const char *name, extern_err_t *err);
/* mode 0: libyaml loader (CLI path, marks); mode 1: serde loader (FFI path) */
int32_t gg_session_add_docs(gg_session *s, const char *const *texts, const size_t *lens, const char *const *names,
                            size_t n, int32_t mode, int32_t nthreads, extern_err_t *err);
/* input parameters (validate -i) merged into every document added after this call; texts are
 * loaded like the CLI's data files (libyaml loader) and merged in order; 0, or the error code */
int32_t gg_session_set_params(gg_session *s, const char *const *texts, const size_t *lens, const char *const *names,
                              size_t n, extern_err_t *err);
int32_t gg_session_upload(gg_session *s, extern_err_t *err);
int32_t gg_session_eval(gg_session *s, int32_t iters, double *ms_out, extern_err_t *err);
char *gg_session_report(gg_session *s, int32_t *exit_code, extern_err_t *err);
char *gg_session_report_format(gg_session *s, int32_t output_format, int32_t *exit_code, extern_err_t *err);
/* the session's HIP device (-1: the process default); before its documents or buffers are on a device */
int32_t gg_session_set_device(gg_session *s, int32_t device);
/* the structured report of documents [first, first + count) alone (count SIZE_MAX: to the end): what a
 * run over just those documents writes -- one rank's shard of a multi-GPU job */
char *gg_session_report_range(gg_session *s, int32_t output_format, size_t first, size_t count, int32_t *exit_code,
                              extern_err_t *err);
/* gg_session_report_range with the report's length in bytes in *len (bulk consumers skip a strlen) */
char *gg_session_report_range_n(gg_session *s, int32_t output_format, size_t first, size_t count, size_t *len,
                                int32_t *exit_code, extern_err_t *err);
/* the report rendered as the shards [0, cuts[0]), [cuts[0], cuts[1]), ... [cuts[ncuts-1], ndocs) and joined
 * as cfn_guard_validate_batch_devices joins its devices' shards (the multi-device join, testable on loaded
 * results without a GPU) */
char *gg_session_report_shards(gg_session *s, int32_t output_format, const size_t *cuts, size_t ncuts, int32_t *exit_code,
                               extern_err_t *err);
/* host-only: the byte-balanced split of cfn_guard_validate_batch_devices -- starts[0..nshards] (starts[k] =
 * first document of shard k, starts[nshards] = n); 0, or -1 for nshards == 0 */
int32_t gg_shard_by_bytes(const size_t *lens, size_t n, size_t nshards, size_t *starts);
int64_t gg_session_stat(gg_session *s, int32_t what);
/* Diagnostic: save an evaluation's results (tiles, rule statuses, records) / load them into a session
 * holding the same rules files and documents (no GPU needed to render its reports). */
int32_t gg_session_save_results(gg_session *s, const char *path, extern_err_t *err);
int32_t gg_session_load_results(gg_session *s, const char *path, extern_err_t *err);
int32_t gg_session_tile_status(gg_session *s, uint8_t *out, size_t n);
double gg_session_last_kernel_ms(gg_session *s);
int32_t gg_device_available(void);
/* Frees the device blocks the library keeps for reuse on `device` (-1: every device).  Freed loader
 * temporaries and session buffers are cached per device (bounded by GG_DEV_CACHE_GB, default 16)
 * because hipFree waits for the whole device to go idle; this hands them back, as
 * torch.cuda.empty_cache() does for torch's allocator.  The streamed entries' page-locked host staging
 * blocks (bounded by GG_PINNED_CACHE_GB per device, default 1) are unpinned and freed too.  Returns the
 * bytes released (device and host). */
int64_t gg_device_cache_release(int32_t device);

/* Asynchronous evaluation on a caller stream (bench.py passes a non-default torch stream).  NULL
 * selects the library's own non-blocking stream -- the legacy default stream cannot be named. */
void gg_session_set_stream(gg_session *s, void *hip_stream);
/* mode 0 (default): one tile per lane, tiles that outgrow the lane heap re-run one tile per
 * wavefront; mode 1: one tile per wavefront for every tile.  lane_heap_bytes 0 keeps 64 KB. */
int32_t gg_session_configure(gg_session *s, int32_t mode, uint32_t lane_heap_bytes);
/* session options (0 = set, -1 = unknown option).  GG_OPT_RX_MEMO_PER_LAUNCH: 1 zeroes the regex
 * is_match memo (2 bits per (pool string, regex), filled by the first evaluation that runs the DFA) before
 * every launch, so each launch pays its own first DFA runs; 0 (default) zeroes it once per upload. */
#define GG_OPT_RX_MEMO_PER_LAUNCH 1
/* GG_OPT_DEFER_RECORDS: 1 leaves the failure records in HBM where the evaluation wrote them at
 * gg_session_fetch (statuses and tallies still come to the host); the device JSON reporter reads them
 * there, and they are compacted and copied down only when a host writer needs them.  0 (default). */
#define GG_OPT_DEFER_RECORDS 2
int32_t gg_session_set_option(gg_session *s, int32_t option, int64_t value);
int32_t gg_session_launch(gg_session *s, extern_err_t *err);  /* enqueue; no host sync */
double gg_session_wait(gg_session *s, extern_err_t *err);     /* kernel ms of the last launch */
int32_t gg_session_fetch(gg_session *s, extern_err_t *err);   /* statuses + records to host */
/* Per (rules file, top rule) x {PASS, FAIL, SKIP, error} u64 tallies of the last launch; index
 * ((file * (max_top + 1) + rule) * 4 + status), rule == max_top is the file-level line.  The
 * device buffer is what the multi-GPU path all-reduces over RCCL. */
size_t gg_session_ncounts(gg_session *s);
void *gg_session_counts_device(gg_session *s);
/* write tallies into a caller-owned device buffer of >= ncounts u64 (NULL: internal buffer) */
void gg_session_bind_counts(gg_session *s, void *dev, size_t n);
/* evaluation-kernel ms of every launch since the last drain (HIP events on the launch stream) */
size_t gg_session_drain_kernel_ms(gg_session *s, double *out, size_t cap, extern_err_t *err);
int32_t gg_session_counts(gg_session *s, uint64_t *out, size_t n);
/* the structured report (json / yaml) of the first max_docs documents (0: all) rendered on the host
 * in document blocks and discarded; returns its size in bytes (end-to-end measurement at sizes whose
 * text would not fit in memory) */
int64_t gg_session_report_bytes(gg_session *s, int32_t output_format, size_t max_docs, int32_t *exit_code,
                                extern_err_t *err);
/* The structured JSON report of the first max_docs documents (0: all) rendered on the session's device
 * (csrc/report_gpu.hip: a size pass and a write pass per block of documents, one lane per document), copied
 * to host memory block by block and discarded; documents the device writer leaves to the host writer
 * (floats, Debug-formatted reasons, map keys / count() values as values) are written by it in place.
 * Returns the report's size in bytes (gg_session_report_bytes' end-to-end measurement, reporter on the
 * device); stats (may be NULL, 8 doubles): device documents, host documents, size-pass ms, write-pass ms,
 * copy-out ms, host-writer ms, body bytes, 0. */
int64_t gg_session_report_json_device(gg_session *s, size_t max_docs, int32_t *exit_code, double *stats, extern_err_t *err);
/* the SARIF report (artifacts + frame on the host, FAILed documents' results rendered on the device), counted */
int64_t gg_session_report_sarif_device(gg_session *s, size_t max_docs, int32_t *exit_code, double *stats, extern_err_t *err);
/* JSON reports of this session (gg_session_report*, the batch entry points): 1 rendered on the device
 * (default, GG_DEVICE_REPORT=0 turns it off), 0 on host threads, -1 back to the environment's choice. */
int32_t gg_session_set_device_report(gg_session *s, int32_t on);
/* diagnostic evaluator counters (nonzero only in the GG_STATS build variant) */
int32_t gg_session_kernel_stats(gg_session *s, uint64_t *out, size_t n);

/* Loader self-check (tests): 1 = JSON fast path builds the libyaml path's exact arena,
 * 0 = they differ, -1 = fast path declined the document. */
int32_t gg_loader_selfcheck(const char *text, size_t len);

/* Host-side diagnostics (no GPU; tests pin the loader and the grammar with them).
 * gg_load_dump: loads one document (mode 0 libyaml / 1 serde, as gg_session_add_docs) and returns a
 * typed rendering of the value tree, e.g. {"check": Bool(true)}; NULL + err on a load error.
 * gg_parse_rules: parses one rules file like parse_rules (validate.rs:658-664); returns 0 = rules,
 * 1 = no rules (Ok(None)), 5 = parse error (err->message = the Error Display). */
char *gg_load_dump(const char *text, size_t len, int32_t mode, extern_err_t *err);
int32_t gg_parse_rules(const char *text, const char *name, extern_err_t *err);
/* sizes of the compiled program (no GPU): out[0] blob words, out[1] words before the regex DFA
 * tables, out[2] regexes, out[3] clauses, out[4] query parts; returns gg_parse_rules' code */
int32_t gg_program_stats(const char *text, const char *name, uint32_t *out);
/* The rule-regex DFA (compiled as for a rules file) run on the host over one haystack: 1 match,
 * 0 no match, -1 unsupported on the MI355X path (look-around, back-references, ...), -2 invalid.
 * stats (may be NULL, 2 values): DFA states, code-point classes; bit 31 of stats[0] set when the regex
 * has no DFA within the limits and runs as the NFA simulation (then NFA states). */
int32_t gg_regex_match(const char *pattern, const char *text, size_t len, uint32_t *stats);

/* Synthetic CloudFormation corpus (BASELINE configs[1]); byte-identical to synth.py cfn_doc. */
size_t gg_synth_cfn_doc(uint64_t index, int32_t n_resources, char *buf, size_t cap);
/* the same template as block-style CloudFormation YAML (byte-identical to synth.py cfn_yaml_doc) */
size_t gg_synth_cfn_yaml_doc(uint64_t index, int32_t n_resources, char *buf, size_t cap);
int32_t gg_session_add_synthetic(gg_session *s, uint64_t first, size_t n, int32_t n_resources, int32_t nthreads,
                                 extern_err_t *err);

/* Device loader (replaces, for strict-JSON input, the reference's
 * Loader::load + PathAwareValue::try_from, guard/src/rules/libyaml/loader.rs:31-195 and
 * guard/src/rules/path_value.rs:414-478, as called from validate.rs:760-787).  Parses and interns
 * the documents on the MI355X into an EMPTY session, building the arena gg_session_add_docs builds.
 * A document outside the device subset (libyaml-only syntax, duplicate keys, nesting past 64, a float
 * beyond the exact fast path, a raw character libyaml reads specially) is built by the host loader
 * and spliced in at its position.  Returns 0 when loaded, 1 when the batch is refused as a whole
 * (a batch-wide limit, or a refused document the host loader rejects too: nothing loaded, err->message
 * says why; gg_session_add_docs reports the loader error), -1 on error.  stats (may be NULL, 10 doubles):
 * kernel ms, nodes, distinct strings, pool bytes, text bytes, H2D ms, D2H ms, intern-table doublings,
 * documents built by the host loader, host text-generation ms (gg_session_add_synthetic_device; else 0).  The loaded nodes stay in HBM for the session's first upload
 * (it packs the device arena from them; only host-built documents cross PCIe again). */
int32_t gg_session_add_docs_device(gg_session *s, const char *const *texts, const size_t *lens, const char *const *names,
                                   size_t n, double *stats, extern_err_t *err);
int32_t gg_session_add_synthetic_device(gg_session *s, uint64_t first, size_t n, int32_t n_resources, int32_t nthreads,
                                        double *stats, extern_err_t *err);
/* gg_session_add_synthetic_device with the corpus written as format 0 JSON or 1 block-style YAML */
int32_t gg_session_add_synthetic_device_fmt(gg_session *s, uint64_t first, size_t n, int32_t n_resources, int32_t nthreads,
                                            int32_t format, double *stats, extern_err_t *err);
/* Host diagnostic: the device loader's float parser (Eisel-Lemire, csrc/eisel_lemire.h) on the JSON
 * number s[0..n): 1 = *out is the correctly rounded double, 0 = refused (its document loads on the host). */
int32_t gg_parse_f64(const char *s, size_t n, double *out);
/* 1 = the device loader builds the host loader's arena (up to string ids), 0 = differs, -1 = refused */
int32_t gg_loader_device_check(const char *const *texts, const size_t *lens, size_t n, extern_err_t *err);

#ifdef __cplusplus
}
#endif

#endif
