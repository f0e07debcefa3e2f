"""Pin the oracle's case-converter query fallback (cruet 0.14.0, eval_context.rs:22,317-325,539-568).

* ``test_with_converter`` restates the reference's own test ``guard/src/rules/eval_context_tests.rs:407-452``:
  a query written in lower case resolves through the converters, and an empty ``Tags`` list gives
  an UnResolved result whose ``traversed_to`` is that list.
* ``test_cruet_published_examples``: the converter functions against the crate's published doc
  examples (cruet is not vendored in the reference; its algorithm is restated in
  oracle/guard_oracle/cruet.py).
"""
from guard_oracle import cruet
from guard_oracle import evaluator as E
from guard_oracle.loader import load_document
from guard_oracle.parser import parse_rules

DOC = """
Resources:
   s3:
     Type: AWS::S3::Bucket
     Properties:
       Tags:
         - Key: 1
           Value: 1
   ec2:
     Type: AWS::EC2::Instance
     Properties:
       ImageId: ami-123456789012
       Tags: []
"""


def test_with_converter():
    rf = parse_rules("let q = resources.*.properties.tags[*].value\n", "t.guard")
    query = rf["assignments"][0]["value"][1]["query"]
    root = E.RootScope(rf, load_document(DOC))
    results = root.query(query)
    assert len(results) == 2  # 2 resources
    kinds = sorted(r[0] for r in results)
    assert kinds == ["R", "U"]
    for r in results:
        if r[0] == "R":
            assert r[1].path == "/Resources/s3/Properties/Tags/0/Value"
            assert r[1].is_scalar()
        else:
            assert r[1].traversed_to.path == "/Resources/ec2/Properties/Tags"


def test_cruet_published_examples():
    assert cruet.to_camel_case("foo_bar") == "fooBar"
    assert cruet.to_camel_case("FooBar") == "fooBar"
    assert cruet.to_pascal_case("foo_bar") == "FooBar"
    assert cruet.to_pascal_case("foo-bar") == "FooBar"
    assert cruet.to_snake_case("FooBar") == "foo_bar"
    assert cruet.to_snake_case("fooBar") == "foo_bar"
    assert cruet.to_kebab_case("FooBar") == "foo-bar"
    assert cruet.to_train_case("foo_bar") == "Foo-Bar"
    assert cruet.to_title_case("foo_bar") == "Foo Bar"
    assert cruet.to_class_case("foo_bars") == "FooBar"
