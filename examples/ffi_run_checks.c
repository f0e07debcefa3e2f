/* guard-ffi consumer built against the MI355X library instead of libcfn_guard_ffi.
 * Same struct layouts and ownership rules as guard-ffi (guard-ffi/src/lib.rs:5-47): the caller
 * frees both the result and err.message on both paths, so free(NULL) must be safe. */
#include <stdio.h>

#include "cfn_guard_mi355x.h"

int main(int argc, char **argv) {
  extern_err_t err = {0, NULL};
  validate_input_t data = {"Resources:\n  b:\n    Type: AWS::S3::Bucket\n    Properties:\n      BucketName: x\n",
                           "template.yaml"};
  validate_input_t rules = {"rule s3_named { Resources.*[ Type == 'AWS::S3::Bucket' ].Properties.BucketName == 'y' }",
                            "s3.guard"};
  char *result = cfn_guard_run_checks(data, rules, 0, &err);
  int code = err.code;
  if (code == 0) {
    fputs(result, stdout);
  } else {
    printf("error: %d (%s)\n", err.code, err.message ? err.message : "");
  }
  cfn_guard_free_string(result);
  cfn_guard_free_string(err.message);
  (void)argc; (void)argv;
  return code == 0 ? 0 : 2;
}
