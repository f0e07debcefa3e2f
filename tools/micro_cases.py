"""Single rule shapes on the cfg-2 corpus (diagnostic; tools/micro.py, tools/kernel_stats.py PACK=micro)."""
CASES = {
    "exists_root": "rule r { Resources exists }",
    "let_typefilter": "let b = Resources.*[ Type == 'AWS::S3::Bucket' ]\nrule r when %b !empty { %b exists }",
    "all_props_exists": "rule r { Resources.*.Properties exists }",
    "all_tags_empty": "rule r { Resources.*.Properties.Tags !empty }",
    "typeblock_1": "rule r { AWS::S3::Bucket { Properties.BucketName exists } }",
    "typeblock_3": "rule r { AWS::S3::Bucket { Properties.BucketName exists\n Properties.VersioningConfiguration exists\n Properties.LoggingConfiguration exists } }",
    "tags_some_regex": "let d = Resources.*[ Type == 'AWS::DynamoDB::Table' ]\nrule r when %d !empty {\n  let p = %d[ some Properties.Tags[*] { Key == /PROD/\n Value == /^App/ } ]\n  %p empty\n}",
    "all_tags_exists": "rule r { Resources.*.Properties.Tags exists }",
    "all_type_eq": "rule r { Resources.*.Type == 'AWS::S3::Bucket' }",
    "var_eq_5": "let b = Resources.*[ Type == 'AWS::S3::Bucket' ]\nrule r when %b !empty {\n" + "\n".join(
        "  %%b.Properties.PublicAccessBlockConfiguration.%s == true" % k for k in
        ["BlockPublicAcls", "BlockPublicPolicy", "IgnorePublicAcls", "RestrictPublicBuckets", "BlockPublicAcls"]) + "\n}",
}
