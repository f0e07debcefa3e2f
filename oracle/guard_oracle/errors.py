"""Error restatement (TEST INFRASTRUCTURE ONLY -- the parity oracle).

Mirrors ``guard/src/rules/errors.rs:9-54`` (thiserror Display strings) and the guard-ffi
error-code table ``guard-ffi/src/errors.rs:12-38``.
"""

_DISPLAY = {
    "JsonError": "Error parsing incoming JSON context {0}",
    "YamlError": "Error parsing incoming YAML context {0}",
    "FormatError": "Formatting error when writing {0}",
    "IoError": "I/O error when reading {0}",
    "ParseError": "Parser Error when parsing `{0}`",
    "RegexError": "Regex expression parse error for rules file {0}",
    "MissingProperty": "Could not evaluate clause for a rule with missing property for incoming context `{0}`",
    "MissingValue": "There was no variable or value object to resolve. Error = `{0}`",
    "RetrievalError": "Could not retrieve data from incoming context. Error = `{0}`",
    "MissingVariable": "Variable assignment could not be resolved in rule file or incoming context `{0}`",
    "MultipleValues": "Conflicting rule or variable assignments inside the same scope `{0}`",
    "IncompatibleRetrievalError": "Types or variable assignments have incompatible types to retrieve `{0}`",
    "IncompatibleError": "Types or variable assignments are incompatible `{0}`",
    "NotComparable": "Comparing incoming context with literals or dynamic results wasn't possible `{0}`",
    "FileNotFoundError": "The path `{0}` does not exist",
    "IllegalArguments": "{0}",
    "InternalError": "{0}",
    "Unsupported": "{0}",
    "Panic": "{0}",   # a Rust panic (unreachable!()): ffi-support code -1, its payload as the message
}

FFI_CODES = {
    "JsonError": 1, "YamlError": 2, "FormatError": 3, "IoError": 4, "ParseError": 5,
    "RegexError": 6, "MissingProperty": 7, "MissingVariable": 8, "MultipleValues": 9,
    "IncompatibleRetrievalError": 10, "IncompatibleError": 11, "NotComparable": 12,
    "ConversionError": 13, "Errors": 14, "RetrievalError": 15, "MissingValue": 16,
    "FileNotFoundError": 17, "IllegalArguments": 18, "XMLError": 20,
}


class GuardError(Exception):
    def __init__(self, kind, msg):
        Exception.__init__(self, msg)
        self.kind = kind
        self.msg = msg

    def display(self):
        return _DISPLAY[self.kind].format(self.msg)

    def __str__(self):
        return self.display()
