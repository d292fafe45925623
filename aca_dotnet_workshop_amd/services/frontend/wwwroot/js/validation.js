// Client-side form validation -- the equivalent of the reference's _ValidationScriptsPartial
// (jquery-validate + jquery-validation-unobtrusive, Pages/Shared/_ValidationScriptsPartial.cshtml,
// rendered by Pages/Tasks/Create.cshtml:45 and Edit.cshtml).  It reads the same unobtrusive
// attributes ASP.NET's tag helpers emit for [Required] / [EmailAddress] / date inputs
// (data-val, data-val-required, data-val-email, data-val-date) and writes messages into the
// matching <span data-valmsg-for="...">, so a form with a missing field is never posted.
// No jQuery: plain DOM, ~60 lines.  The server-side binder (services/frontend/app.py _bind)
// still validates every post, exactly like ModelState in the reference.
(function (root) {
  "use strict";

  var EMAIL = /^[^\s@]+@[^\s@]+$/;
  var DATE = /^\d{4}-\d{2}-\d{2}$/;

  // Returns the first failing rule's message for `value` under the element's data-val-* rules,
  // or "" when the value is valid.  `attr(name)` reads an attribute (testable without a DOM).
  function check(value, attr) {
    if (attr("data-val") !== "true") return "";
    var v = (value || "").trim();
    if (attr("data-val-required") !== null && v === "") return attr("data-val-required");
    if (v === "") return "";
    if (attr("data-val-email") !== null && !EMAIL.test(v)) return attr("data-val-email");
    if (attr("data-val-date") !== null && (!DATE.test(v) || isNaN(Date.parse(v)))) return attr("data-val-date");
    return "";
  }

  function show(form, input, msg) {
    var span = form.querySelector('[data-valmsg-for="' + input.name + '"]');
    if (span) {
      span.textContent = msg;
      span.className = msg ? "field-validation-error text-danger" : "field-validation-valid text-danger";
    }
    input.classList.toggle("input-validation-error", !!msg);
    input.setAttribute("aria-invalid", msg ? "true" : "false");
  }

  function validateInput(form, input) {
    var msg = check(input.value, function (n) { return input.getAttribute(n); });
    show(form, input, msg);
    return !msg;
  }

  function attach(form) {
    var inputs = form.querySelectorAll('[data-val="true"]');
    form.setAttribute("novalidate", "novalidate");  // our messages instead of the browser's bubbles
    form.addEventListener("submit", function (ev) {
      var ok = true, first = null;
      for (var i = 0; i < inputs.length; i++) {
        if (!validateInput(form, inputs[i])) {
          ok = false;
          first = first || inputs[i];
        }
      }
      if (!ok) {
        ev.preventDefault();
        if (first && first.focus) first.focus();
      }
    });
    for (var i = 0; i < inputs.length; i++) {
      (function (input) {
        input.addEventListener("blur", function () { validateInput(form, input); });
        input.addEventListener("input", function () {
          if (input.classList.contains("input-validation-error")) validateInput(form, input);
        });
      })(inputs[i]);
    }
  }

  if (typeof module !== "undefined" && module.exports) module.exports = { check: check };
  if (root.document) {
    var forms = root.document.querySelectorAll("form");
    for (var i = 0; i < forms.length; i++) attach(forms[i]);
  }
})(typeof window !== "undefined" ? window : {});
