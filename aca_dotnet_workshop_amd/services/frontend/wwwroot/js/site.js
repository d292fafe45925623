// Site-wide scripts (intentionally empty, like the reference's wwwroot/js/site.js).
