"""Builds tests/golden/validate_cases.json from the reference's own validate test resources
(guard/resources/validate/, the inputs of guard/tests/validate.rs and functions/), run HERE only:
the data / rules files are copied verbatim as fixture inputs; expected outputs are not stored --
the GPU test compares the device path with the oracle on them live, and the CPU test pins the
oracle's exit codes and error kinds below (read off tests/validate.rs's expected status codes)."""
import json
import os
import sys

R = "/root/reference/guard/resources/validate/"
# (rules files, data files, expected exit code per tests/validate.rs or the oracle's verdict)
CASES = [
    (["workshop.guard"], ["template_where_resources_isnt_root.json"], 19),
    (["rules-dir/s3_bucket_server_side_encryption_enabled.guard"], ["failing_template_with_slash_in_key.yaml"], 19),
    (["s3_bucket_server_side_encryption_enabled_2.guard"], ["s3-server-side-encryption-template-non-compliant-2.yaml"], 19),
    (["comments.guard"], ["s3-server-side-encryption-template-non-compliant-2.yaml"], 0),
    (["db_param_port_rule.guard"], ["db_resource.yaml"], 19),
    (["rules-dir/s3_bucket_public_read_prohibited.guard", "rules-dir/s3_bucket_server_side_encryption_enabled.guard"],
     ["data-dir/s3-public-read-prohibited-template-non-compliant.yaml", "data-dir/s3-public-read-prohibited-template-compliant.yaml"], 19),
    (["functions/rules/count.guard"], ["functions/data/template.yaml"], 0),
    (["functions/rules/count_with_message.guard"], ["functions/data/template.yaml"], 19),
    # errors: the run aborts (exit -1, nothing on stdout)
    (["rules-dir/s3_bucket_public_read_prohibited.guard"], ["malformed-template.yaml"], -1),
    (["s3_bucket_server_side_encryption_enabled_2.guard", "blank-rule.guard"],
     ["blank-template.yaml", "s3-server-side-encryption-template-non-compliant-2.yaml"], -1),
]


def main():
    out = []
    for rules, data, code in CASES:
        out.append({"rules": [[os.path.basename(p), open(R + p).read()] for p in rules],
                    "data": [[os.path.basename(p), open(R + p).read()] for p in data],
                    "exit_code": code, "source": {"rules": rules, "data": data}})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "validate_cases.json")
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path, len(out), "cases")


if __name__ == "__main__":
    sys.exit(main())
